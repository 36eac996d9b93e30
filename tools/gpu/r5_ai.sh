# Round 5 (ai): a block's skip-conv weight gradient launched after the block's units
# (XCP_SKIP_WGRAD_LATE=1) vs before them (default): engine grad test, in-step A/B, 3 rounds
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
XCP_SKIP_WGRAD_LATE=1 timeout -k 10 300 python -u -m pytest -p no:cacheprovider --timeout 200 --timeout-method thread -rf -x -q tests/test_gpu_model.py -k "backbone64 or deterministic or bench_size" > gpurun_out/ai_tests.log 2>&1 || exit $?
for r in 1 2 3; do
  timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 > gpurun_out/ai_old_$r.log 2> gpurun_out/ai_old_$r.err || exit $?
  XCP_SKIP_WGRAD_LATE=1 timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 > gpurun_out/ai_new_$r.log 2> gpurun_out/ai_new_$r.err || exit $?
done
