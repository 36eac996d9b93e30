# Round 5 (af): weight gradient before input gradient as the default: full GPU suite, in-step A/B
# XCP_WGRAD_FIRST=0 / default, 3 rounds (confirmation on a second box)
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
T="python -u -m pytest -p no:cacheprovider --timeout 200 --timeout-method thread -rf"
timeout -k 10 400 $T -x -q -m gpu tests > gpurun_out/af_suite.log 2>&1 || exit $?
for r in 1 2 3; do
  XCP_WGRAD_FIRST=0 timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 > gpurun_out/af_off_$r.log 2> gpurun_out/af_off_$r.err || exit $?
  timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 > gpurun_out/af_on_$r.log 2> gpurun_out/af_on_$r.err || exit $?
done
