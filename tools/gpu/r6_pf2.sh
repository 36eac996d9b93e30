# Round 6: gemm_nt256p_kernel's two-K-tile prefetch at tile boundaries (XCP_NT_PF2=1): NT tests with it on,
# per-shape A/B (tools/nt_env_ab.py), then the step (default bench line) interleaved off / on
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
( while true; do date >> gpurun_out/pf2_heartbeat.txt; sleep 50; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
XCP_NT_PF2=1 timeout -k 10 400 python -u -m pytest -p no:cacheprovider --timeout 200 --timeout-method thread -x -q tests/test_gpu_kernels.py -k "gemm_nt or sep_fwd or unit" > gpurun_out/pf2_tests.log 2>&1 || exit $?
timeout -k 10 400 python -u tools/nt_env_ab.py 3 XCP_NT_PF2=0,1 > gpurun_out/pf2_ab.txt 2>&1 || exit $?
for r in 1 2; do
for v in 0 1; do
  echo "== XCP_NT_PF2=$v" >> gpurun_out/pf2_step.txt
  XCP_NT_PF2=$v timeout -k 10 200 python bench.py --cpu-baseline off --steps 20 --warmup 5 --measured-peaks off > gpurun_out/pf2_one.json 2>> gpurun_out/pf2_step.err || exit $?
  grep '^{' gpurun_out/pf2_one.json | python -c "import sys,json; d=json.loads(sys.stdin.read().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['roofline']['achieved'], d['roofline']['frac'])" >> gpurun_out/pf2_step.txt || exit $?
done; done
