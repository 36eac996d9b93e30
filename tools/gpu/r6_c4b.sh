# Round 6: the fused block1 forward's width gate (engine.SEP_MIN_W): C4 / C5 / C2 lines with the gate
# (default) and with every supported width fused (XCP_SEP_NARROW=1), interleaved; sep_fwd kernel tests
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
( while true; do date >> gpurun_out/c4b_heartbeat.txt; sleep 50; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
timeout -k 10 300 python -u -m pytest -p no:cacheprovider --timeout 200 --timeout-method thread -x -q tests/test_gpu_kernels.py -k "sep_fwd" > gpurun_out/c4b_tests.log 2>&1 || exit $?
for r in 1 2; do
for m in lstma auface xception; do
for v in "" XCP_SEP_NARROW=1; do
  echo "== $m $v" >> gpurun_out/c4b_ab.txt
  env $v timeout -k 10 200 python bench.py --model $m --cpu-baseline off --steps 10 --warmup 3 > gpurun_out/c4b_one.json 2>> gpurun_out/c4b_ab.err || exit $?
  grep '^{' gpurun_out/c4b_one.json | python -c "import sys,json; d=json.loads(sys.stdin.read().splitlines()[-1]); f=d.get('diag',{}).get('frozen',{}) or {}; print(d['value'], d['ms_per_step'], f.get('fwd_ms'), f.get('bwd_ms'))" >> gpurun_out/c4b_ab.txt || exit $?
done; done; done
cp gpurun_out/c4b_one.json gpurun_out/c4b_last.json
