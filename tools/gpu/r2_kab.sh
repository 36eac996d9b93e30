# GPU: targeted kernel tests, then a kbench A/B of the current library vs tools/exp/old/libxcp.so
# (new, old, new in one run).  usage: bash tools/gpu/r2_kab.sh "<kbench names>" ["<pytest -k expr>"]
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
if [ -n "$2" ]; then
  timeout -k 10 170 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -k "$2" > gpurun_out/kab_tests.log 2>&1 || exit $?
fi
timeout -k 10 170 python -u tools/kbench.py $1 > gpurun_out/kab_new1.log 2>&1 || exit $?
cp multimodal-deepfake-detection_amd/xcp/libxcp.so /tmp/libxcp_new.so
cp tools/exp/old/libxcp.so multimodal-deepfake-detection_amd/xcp/libxcp.so
timeout -k 10 170 python -u tools/kbench.py $1 > gpurun_out/kab_old.log 2>&1 || exit $?
cp /tmp/libxcp_new.so multimodal-deepfake-detection_amd/xcp/libxcp.so
timeout -k 10 170 python -u tools/kbench.py $1 > gpurun_out/kab_new2.log 2>&1
