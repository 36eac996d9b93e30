# GPU: pooled-tail micro-benchmark, current library vs the previous bn.hip (A/B in one run).
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 170 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -k "tail or maxpool" > gpurun_out/r2_tail_tests.log 2>&1 || exit $?
timeout -k 10 200 python -u tools/kbench.py tailpool > gpurun_out/r2_tail_new1.log 2>&1 || exit $?
cp multimodal-deepfake-detection_amd/xcp/libxcp.so /tmp/libxcp_new.so
cp tools/exp/old/libxcp.so multimodal-deepfake-detection_amd/xcp/libxcp.so
timeout -k 10 200 python -u tools/kbench.py tailpool > gpurun_out/r2_tail_old.log 2>&1 || exit $?
cp /tmp/libxcp_new.so multimodal-deepfake-detection_amd/xcp/libxcp.so
timeout -k 10 200 python -u tools/kbench.py tailpool > gpurun_out/r2_tail_new2.log 2>&1
