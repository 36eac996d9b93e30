# Round 6: the 256p NT kernel's last K-tile on its first 32-deep half only when K % 64 <= 32 (XCP_NT_KHALF, default
# on): bitwise tests, the op alone (kbench gemm / roof_ops), then the step A/B, order rotated
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_kernels.py -k "gemm_nt" > gpurun_out/khalf_tests.txt 2>&1 || exit $?
for f in 0 1 0 1; do
  echo "== XCP_NT_KHALF=$f" >> gpurun_out/khalf_kb.txt
  XCP_NT_KHALF=$f timeout -k 10 120 python -u tools/kbench.py gemm >> gpurun_out/khalf_kb.txt 2>&1 || exit $?
done
A="XCP_NT_KHALF=1"; B="XCP_NT_KHALF=0"
for order in "A B" "B A" "A B" "B A"; do
for k in $order; do
  v=${!k}
  echo "== $v" >> gpurun_out/khalf_ab.txt
  env $v timeout -k 10 200 python bench.py --cpu-baseline off --steps 20 --warmup 5 --measured-peaks off --diag off > gpurun_out/khalf_one.json 2>> gpurun_out/khalf_ab.err || exit $?
  grep '^{' gpurun_out/khalf_one.json | python -c "import sys,json; d=json.loads(sys.stdin.read().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['roofline']['achieved'])" >> gpurun_out/khalf_ab.txt || exit $?
done; done
