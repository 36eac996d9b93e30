# Round 5 (a): the new parity tests first (T = 120 recurrence, capturable Adam with a late parameter,
# 2-rank DDP with the async buffer broadcast), then the whole GPU suite, then the default bench line
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
T="python -u -m pytest -p no:cacheprovider --timeout 300 --timeout-method thread -rf"
timeout -k 10 600 $T -v tests -m gpu -k "t120 or late_parameter or two_rank" > gpurun_out/a_new.log 2>&1 || exit $?
timeout -k 10 1500 $T -q tests -m gpu > gpurun_out/a_suite.log 2>&1 || exit $?
timeout -k 10 300 python bench.py > gpurun_out/a_bench.json 2> gpurun_out/a_bench.err || exit $?
