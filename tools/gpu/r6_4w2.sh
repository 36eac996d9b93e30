# Round 6: gemm_nt4w_kernel with each step's 8-MFMA groups fenced beside their DMA piece and fragment reads
# (XCP_NT_4W=2): NT tests with it on, per-shape A/B against the default, the step once each
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
( while true; do date >> gpurun_out/w42_heartbeat.txt; sleep 50; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
XCP_NT_4W=2 timeout -k 10 400 python -u -m pytest -p no:cacheprovider --timeout 200 --timeout-method thread -x -q tests/test_gpu_kernels.py -k "gemm_nt" > gpurun_out/w42_tests.log 2>&1 || exit $?
timeout -k 10 400 python -u tools/nt_env_ab.py 3 XCP_NT_4W=0,2 > gpurun_out/w42_ab.txt 2>&1 || exit $?
for v in 0 2; do
  echo "== XCP_NT_4W=$v" >> gpurun_out/w42_step.txt
  XCP_NT_4W=$v timeout -k 10 200 python bench.py --cpu-baseline off --steps 20 --warmup 5 --measured-peaks off > gpurun_out/w42_one.json 2>> gpurun_out/w42_step.err || exit $?
  grep '^{' gpurun_out/w42_one.json | python -c "import sys,json; d=json.loads(sys.stdin.read().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['roofline']['achieved'], d['roofline']['frac'])" >> gpurun_out/w42_step.txt || exit $?
done
