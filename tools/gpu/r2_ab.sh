# GPU: targeted tests, then bench A/B of the current library vs tools/exp/old/libxcp.so in one run.
# usage: bash tools/gpu/r2_ab.sh "<pytest -k expr>"
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
if [ -n "$1" ]; then
  timeout -k 10 170 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -k "$1" > gpurun_out/ab_tests.log 2>&1 || exit $?
fi
timeout -k 10 170 python -u bench.py --steps 20 --warmup 5 --cpu-baseline off > gpurun_out/ab_new1.json 2> gpurun_out/ab_new1.err || exit $?
cp multimodal-deepfake-detection_amd/xcp/libxcp.so /tmp/libxcp_new.so
cp tools/exp/old/libxcp.so multimodal-deepfake-detection_amd/xcp/libxcp.so
timeout -k 10 170 python -u bench.py --steps 20 --warmup 5 --cpu-baseline off > gpurun_out/ab_old.json 2> gpurun_out/ab_old.err || exit $?
cp /tmp/libxcp_new.so multimodal-deepfake-detection_amd/xcp/libxcp.so
timeout -k 10 170 python -u bench.py --steps 20 --warmup 5 --cpu-baseline off > gpurun_out/ab_new2.json 2> gpurun_out/ab_new2.err
