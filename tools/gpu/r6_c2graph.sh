# Round 6: the C2 line (Xception, 64 frames) replayed as one HIP graph vs eager launches, interleaved
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for r in 1 2 3 4; do
for v in off on; do
  echo "== --graph $v" >> gpurun_out/c2graph.txt
  timeout -k 10 200 python -u bench.py --model xception --cpu-baseline off --graph $v > gpurun_out/c2graph_one.json 2>> gpurun_out/c2graph.err || exit $?
  grep '^{' gpurun_out/c2graph_one.json | python -c "import sys,json; d=json.loads(sys.stdin.read().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['loss'], d['diag']['unfrozen']['step_ms'])" >> gpurun_out/c2graph.txt || exit $?
done; done
