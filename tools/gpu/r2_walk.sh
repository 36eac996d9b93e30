# GPU: depthwise row-walk kernels -- dw parity tests, then kbench fwd/bwd shapes for the current
# library and tools/exp/old/libxcp.so (previous kernels) in one run.
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_kernels.py -k "dw" > gpurun_out/walk_tests.log 2>&1 || exit $?
timeout -k 10 200 python -u tools/kbench.py copy dwshapes dwbshapes > gpurun_out/walk_new.log 2>&1 || exit $?
cp multimodal-deepfake-detection_amd/xcp/libxcp.so /tmp/libxcp_new.so
cp tools/exp/old/libxcp.so multimodal-deepfake-detection_amd/xcp/libxcp.so
timeout -k 10 200 python -u tools/kbench.py copy dwshapes dwbshapes > gpurun_out/walk_old.log 2>&1
rc=$?
cp /tmp/libxcp_new.so multimodal-deepfake-detection_amd/xcp/libxcp.so
exit $rc
