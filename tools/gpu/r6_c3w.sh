# Round 6: stem conv2 weight gradient, shifted-gradient forms (XCP_CONV3_WGRAD=1/2) vs the nine-X-fragment form (0):
# the forms' parity tests, the kernel alone (kbench conv2), then the step interleaved
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -k "conv3x3" > gpurun_out/c3w_tests.txt 2>&1 || exit $?
for f in 0 1 2; do
  echo "== form $f" >> gpurun_out/c3w_kb.txt
  XCP_CONV3_WGRAD=$f timeout -k 10 120 python -u tools/kbench.py conv2 >> gpurun_out/c3w_kb.txt 2>&1 || exit $?
done
for r in 1 2 3; do
for f in 0 2 1; do
  echo "== XCP_CONV3_WGRAD=$f" >> gpurun_out/c3w_ab.txt
  XCP_CONV3_WGRAD=$f timeout -k 10 200 python bench.py --cpu-baseline off --steps 20 --warmup 5 --measured-peaks off --diag off > gpurun_out/c3w_one.json 2>> gpurun_out/c3w_ab.err || exit $?
  grep '^{' gpurun_out/c3w_one.json | python -c "import sys,json; d=json.loads(sys.stdin.read().splitlines()[-1]); print(d['value'], d['ms_per_step'])" >> gpurun_out/c3w_ab.txt || exit $?
done; done
