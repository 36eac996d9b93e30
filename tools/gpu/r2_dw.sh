# GPU: depthwise parity tests, then dw_fwd timings for the built library and a 5-WG/CU variant.
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py -k "dw" -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/r2_dw_t.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/r2_dw_t.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u tools/kbench.py copy dw_fwd > gpurun_out/r2_dw_b4.log 2>&1 || exit $?
cp tools/exp/v5/libxcp.so multimodal-deepfake-detection_amd/xcp/libxcp.so
timeout -k 10 200 python -u tools/kbench.py dw_fwd > gpurun_out/r2_dw_b5.log 2>&1
