# Round 6: the stem backward's BN1 sums (chanred, 520 us in the step) wait behind the side stream's conv2 weight
# gradient (792 us, every CU).  A/B of the conv2 weight gradient launched before conv2's input gradient (default,
# XCP_STEM_WGRAD_EARLY=1) vs after BN1's coefficients (=0), and the side stream at low priority, interleaved
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
( while true; do date >> gpurun_out/stem_heartbeat.txt; sleep 50; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
for r in 1 2 3; do
for v in "XCP_STEM_WGRAD_EARLY=1" "XCP_STEM_WGRAD_EARLY=0" "XCP_SIDE_PRIO=low"; do
  echo "== $v" >> gpurun_out/stem_ab.txt
  env $v timeout -k 10 200 python bench.py --cpu-baseline off --steps 20 --warmup 5 --measured-peaks off --diag off > gpurun_out/stem_one.json 2>> gpurun_out/stem_ab.err || exit $?
  grep '^{' gpurun_out/stem_one.json | python -c "import sys,json; d=json.loads(sys.stdin.read().splitlines()[-1]); print(d['value'], d['ms_per_step'])" >> gpurun_out/stem_ab.txt || exit $?
done; done
