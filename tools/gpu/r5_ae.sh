# Round 5 (ae): a unit's weight gradient launched before its input gradient (XCP_WGRAD_FIRST=1) vs after:
# model tests under the flag, in-step A/B, 3 rounds
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
T="python -u -m pytest -p no:cacheprovider --timeout 200 --timeout-method thread -rf"
XCP_WGRAD_FIRST=1 timeout -k 10 400 $T -x -q -m gpu tests/test_gpu_model.py tests/test_gpu_train_step.py > gpurun_out/ae_tests.log 2>&1 || exit $?
for r in 1 2 3; do
  XCP_WGRAD_FIRST=0 timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 > gpurun_out/ae_off_$r.log 2> gpurun_out/ae_off_$r.err || exit $?
  XCP_WGRAD_FIRST=1 timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 > gpurun_out/ae_on_$r.log 2> gpurun_out/ae_on_$r.err || exit $?
done
