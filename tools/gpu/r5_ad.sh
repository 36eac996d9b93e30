# Round 5 (ad): the NT tile-queue test (repeated launches, two streams)
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest -p no:cacheprovider --timeout 200 --timeout-method thread -rf -x -q tests/test_gpu_kernels.py -k "tile_queue or persistent" > gpurun_out/ad_tests.log 2>&1 || exit $?
