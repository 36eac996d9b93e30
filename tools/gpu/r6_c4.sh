# Round 6: the C4 (XceptionLSTMA frozen) line fell from 2146 clips/s (r03) to ~1830 (r06); forward 6.08 -> 7.34 ms.
# Kernel trace of the line at HEAD + env A/Bs of the forward forms added in rounds 4-6.
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
( while true; do date >> gpurun_out/c4_heartbeat.txt; sleep 50; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
L="python bench.py --model lstma --cpu-baseline off --steps 5 --warmup 2"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_c4 -o kt -- $L > gpurun_out/c4_prof.log 2>&1 || exit $?
python tools/prof_summary.py gpurun_out/prof_c4 60 > gpurun_out/c4_kernels.txt 2>&1
find gpurun_out/prof_c4 -name "*.csv" -size +2M -delete 2>/dev/null || true
for v in "" XCP_LSTM_PERSIST=0 XCP_SEP_FUSED=0 XCP_STEM_FUSED=0 XCP_NT_ONESHOT=1 XCP_CONV2_ACTIN=0 XCP_PAD_728=0; do
  echo "== $v" >> gpurun_out/c4_ab.txt
  env $v timeout -k 10 200 python bench.py --model lstma --cpu-baseline off --steps 10 --warmup 3 > gpurun_out/c4_one.json 2>> gpurun_out/c4_ab.err || exit $?
  grep '^{' gpurun_out/c4_one.json | python -c "import sys,json; d=json.loads(sys.stdin.read().splitlines()[-1]); f=d['diag'].get('frozen',{}); print(d['value'], d['ms_per_step'], f.get('fwd_ms'), f.get('bwd_ms'))" >> gpurun_out/c4_ab.txt || exit $?
done
