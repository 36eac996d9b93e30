# Round 6: stem conv2 weight gradient default = shifted form 1.  Kernel trace of the step (stem tail layout), then
# A/B of the conv2 weight gradient on the side stream (default) vs the main stream after BN1's sums (XCP_STEM_WGRAD_SIDE=0)
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_c3w -o kt -- python -u bench.py --steps 5 --warmup 2 --cpu-baseline off --measured-peaks off --diag off > gpurun_out/c3w2_prof.log 2>&1 || exit $?
for r in 1 2 3; do
for v in "XCP_STEM_WGRAD_SIDE=1" "XCP_STEM_WGRAD_SIDE=0" "XCP_CONV3_WGRAD=0"; do
  echo "== $v" >> gpurun_out/c3w2_ab.txt
  env $v timeout -k 10 200 python bench.py --cpu-baseline off --steps 20 --warmup 5 --measured-peaks off --diag off > gpurun_out/c3w2_one.json 2>> gpurun_out/c3w2_ab.err || exit $?
  grep '^{' gpurun_out/c3w2_one.json | python -c "import sys,json; d=json.loads(sys.stdin.read().splitlines()[-1]); print(d['value'], d['ms_per_step'])" >> gpurun_out/c3w2_ab.txt || exit $?
done; done
