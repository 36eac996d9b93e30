# Round 6: stem conv2 weight gradient launched before conv2's input gradient (default, XCP_STEM_WGRAD_EARLY=1, with the
# narrow BN1 finalize beside it) vs after BN1's coefficients (=0), with the shifted weight-gradient form; order rotated
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
A="XCP_STEM_WGRAD_EARLY=1"; B="XCP_STEM_WGRAD_EARLY=0"
for order in "A B" "B A" "A B" "B A" "A B" "B A"; do
for k in $order; do
  v=${!k}
  echo "== $v" >> gpurun_out/early_ab.txt
  env $v timeout -k 10 200 python bench.py --cpu-baseline off --steps 20 --warmup 5 --measured-peaks off --diag off > gpurun_out/early_one.json 2>> gpurun_out/early_ab.err || exit $?
  grep '^{' gpurun_out/early_one.json | python -c "import sys,json; d=json.loads(sys.stdin.read().splitlines()[-1]); print(d['value'], d['ms_per_step'])" >> gpurun_out/early_ab.txt || exit $?
done; done
