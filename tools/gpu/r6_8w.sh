# Round 6: gemm_nt8w_kernel (8 waves, 128x64 each, on the 4-slot ring of 32-deep steps, one barrier per step,
# continuous fill across tiles; XCP_NT_8W=1): NT tests with it on, per-shape A/B, then the step
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
( while true; do date >> gpurun_out/w8_heartbeat.txt; sleep 50; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
timeout -k 10 300 python -u -m pytest -p no:cacheprovider --timeout 120 --timeout-method thread -x -q tests/test_gpu_kernels.py -k "half_tiles_bitwise and 8W" > gpurun_out/w8_tests0.log 2>&1 || exit $?
XCP_NT_8W=1 timeout -k 10 400 python -u -m pytest -p no:cacheprovider --timeout 200 --timeout-method thread -x -q tests/test_gpu_kernels.py -k "gemm_nt or sep_fwd or unit" > gpurun_out/w8_tests.log 2>&1 || exit $?
timeout -k 10 400 python -u tools/nt_env_ab.py 3 XCP_NT_8W=0,1 > gpurun_out/w8_ab.txt 2>&1 || exit $?
for r in 1 2; do
for v in 0 1; do
  echo "== XCP_NT_8W=$v" >> gpurun_out/w8_step.txt
  XCP_NT_8W=$v timeout -k 10 200 python bench.py --cpu-baseline off --steps 20 --warmup 5 --measured-peaks off > gpurun_out/w8_one.json 2>> gpurun_out/w8_step.err || exit $?
  grep '^{' gpurun_out/w8_one.json | python -c "import sys,json; d=json.loads(sys.stdin.read().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['roofline']['achieved'], d['roofline']['frac'])" >> gpurun_out/w8_step.txt || exit $?
done; done
