# Round 6: is the headline step launch-bound (host issue time per step vs device time), and the one-graph
# replay (--graph on) of the headline step against eager launches, interleaved; the C4 line likewise
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
( while true; do date >> gpurun_out/host_heartbeat.txt; sleep 50; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
timeout -k 10 300 python -u tools/cpu_launch_probe.py 10 > gpurun_out/host_probe.txt 2>&1 || exit $?
for r in 1 2; do
for v in off on; do
  echo "== lstmv graph $v" >> gpurun_out/host_graph.txt
  timeout -k 10 300 python bench.py --cpu-baseline off --steps 20 --warmup 5 --measured-peaks off --graph $v > gpurun_out/host_one.json 2>> gpurun_out/host_graph.err || exit $?
  grep '^{' gpurun_out/host_one.json | python -c "import sys,json; d=json.loads(sys.stdin.read().splitlines()[-1]); print(d['value'], d['ms_per_step'])" >> gpurun_out/host_graph.txt || exit $?
done; done
