# Round 6: the C4 line after the width gate: kernel trace + stream timeline; one-graph replay A/B
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
( while true; do date >> gpurun_out/c4c_heartbeat.txt; sleep 50; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
L="python bench.py --model lstma --cpu-baseline off --steps 5 --warmup 2 --measured-peaks off --diag off"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_c4c -o kt -- $L > gpurun_out/c4c_prof.log 2>&1 || exit $?
python tools/prof_summary.py gpurun_out/prof_c4c 60 > gpurun_out/c4c_kernels.txt 2>&1
python tools/stream_timeline.py "$(find gpurun_out/prof_c4c -name "*kernel_trace.csv" | head -1)" 40 > gpurun_out/c4c_timeline.txt 2>&1
find gpurun_out/prof_c4c -name "*.csv" -size +2M -delete 2>/dev/null || true
for r in 1 2; do
for v in off on; do
  echo "== graph $v" >> gpurun_out/c4c_ab.txt
  timeout -k 10 200 python bench.py --model lstma --cpu-baseline off --steps 20 --warmup 5 --graph $v > gpurun_out/c4c_one.json 2>> gpurun_out/c4c_ab.err || exit $?
  grep '^{' gpurun_out/c4c_one.json | python -c "import sys,json; d=json.loads(sys.stdin.read().splitlines()[-1]); print(d['value'], d['ms_per_step'])" >> gpurun_out/c4c_ab.txt || exit $?
done; done
