# Round 6: the middle-flow weight gradient (TN, side stream, half the CUs) overlaps the next unit's input-gradient
# GEMM (NT 133 us alone, ~190 us beside TN).  A/B: TN(u) launched after NT(u+1) (XCP_WGRAD_DEFER=1), with the
# side stream's share at half / all of the CUs (XCP_TN_TARGET_WGS), interleaved; the schedule test first.
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_train_step.py -k wgrad_schedule > gpurun_out/defer_test.txt 2>&1 || exit $?
for r in 1 2 3; do
for v in "XCP_WGRAD_DEFER=0" "XCP_WGRAD_DEFER=1" "XCP_WGRAD_DEFER=1 XCP_TN_TARGET_WGS=256" "XCP_TN_TARGET_WGS=256"; do
  echo "== $v" >> gpurun_out/defer_ab.txt
  env $v timeout -k 10 200 python bench.py --cpu-baseline off --steps 20 --warmup 5 --measured-peaks off --diag off > gpurun_out/defer_one.json 2>> gpurun_out/defer_ab.err || exit $?
  grep '^{' gpurun_out/defer_one.json | python -c "import sys,json; d=json.loads(sys.stdin.read().splitlines()[-1]); print(d['value'], d['ms_per_step'])" >> gpurun_out/defer_ab.txt || exit $?
done; done
