# Round 6: the clip-grouped persistent LSTM backward at two clips per wave (XCP_LSTM_BWD=cg2, 256 workgroups at B 16 x H 512)
# tests with it on, the recurrence A/B (tools/lstm_ab.py), the C4 line default vs the persistent backward cg2
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
( while true; do date >> gpurun_out/cg2_heartbeat.txt; sleep 50; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
timeout -k 10 300 python -u -m pytest -p no:cacheprovider --timeout 200 --timeout-method thread -x -q tests/test_gpu_kernels.py -k "lstm_bwd_clip_grouped" > gpurun_out/cg2_tests0.log 2>&1 || exit $?
XCP_LSTM_BWD=cg2 XCP_LSTM_PERSIST=1 timeout -k 10 300 python -u -m pytest -p no:cacheprovider --timeout 200 --timeout-method thread -x -q tests/test_gpu_kernels.py -k "lstm" > gpurun_out/cg2_tests.log 2>&1 || exit $?
timeout -k 10 300 python -u tools/lstm_ab.py 3 > gpurun_out/cg2_ab.txt 2>&1 || exit $?
for r in 1 2; do
for v in default cg; do
  echo "== $v" >> gpurun_out/cg2_c4.txt
  if [ $v = cg ]; then export XCP_LSTM_PERSIST=1 XCP_LSTM_BWD=cg2; else unset XCP_LSTM_PERSIST XCP_LSTM_BWD; fi
  timeout -k 10 200 python bench.py --model lstma --cpu-baseline off --steps 20 --warmup 5 > gpurun_out/cg2_one.json 2>> gpurun_out/cg2_c4.err || exit $?
  grep '^{' gpurun_out/cg2_one.json | python -c "import sys,json; d=json.loads(sys.stdin.read().splitlines()[-1]); print(d['value'], d['ms_per_step'])" >> gpurun_out/cg2_c4.txt || exit $?
done; done
