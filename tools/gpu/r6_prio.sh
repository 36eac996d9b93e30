# Round 6: main stream above the weight-gradient stream at the dispatcher (XCP_BENCH_MAIN_PRIO=high: the run on a
# greatest-priority stream; the side stream stays at the default = least priority), with the weight-gradient GEMM on
# half / every CU / more, shorter workgroups (XCP_TN_TARGET_WGS); order rotated per repetition
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
A="XCP_BENCH_MAIN_PRIO=none"; B="XCP_BENCH_MAIN_PRIO=high"; C="XCP_BENCH_MAIN_PRIO=high XCP_TN_TARGET_WGS=256"; D="XCP_BENCH_MAIN_PRIO=high XCP_TN_TARGET_WGS=512"
for order in "A B C D" "B C D A" "C D A B"; do
for k in $order; do
  v=${!k}
  echo "== $v" >> gpurun_out/prio_ab.txt
  env $v timeout -k 10 200 python bench.py --cpu-baseline off --steps 20 --warmup 5 --measured-peaks off --diag off > gpurun_out/prio_one.json 2>> gpurun_out/prio_ab.err || exit $?
  grep '^{' gpurun_out/prio_one.json | python -c "import sys,json; d=json.loads(sys.stdin.read().splitlines()[-1]); print(d['value'], d['ms_per_step'])" >> gpurun_out/prio_ab.txt || exit $?
done; done
