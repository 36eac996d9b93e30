# Round 6 (a): full GPU suite after the ADVICE fixes (sepfwd counted wait, plain dw-backward ring reads on
# every form, DDP buffer waits) and the C5 reference-shape test; smoke; one bench line
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
T="python -u -m pytest -p no:cacheprovider --timeout 200 --timeout-method thread -rf"
timeout -k 10 600 $T -x -q -m gpu tests/ --durations=15 > gpurun_out/a_gputests.log 2>&1 || exit $?
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/a_smoke.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py > gpurun_out/a_bench.log 2> gpurun_out/a_bench.err || exit $?
