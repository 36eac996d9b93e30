# Round 6: the C2 line (Xception, 64 frames) -- v5 record showed erratic steps (11.97 .. 19.07 ms); re-measure with the
# stem forms A/B (XCP_CONV3_WGRAD=0 + XCP_STEM_FIN_NARROW=0 = v4 stem), interleaved
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for r in 1 2 3; do
for v in "XCP_STEM_FIN_NARROW=1" "XCP_CONV3_WGRAD=0 XCP_STEM_FIN_NARROW=0"; do
  echo "== $v" >> gpurun_out/c2chk.txt
  env $v timeout -k 10 200 python -u bench.py --model xception --cpu-baseline off > gpurun_out/c2chk_one.json 2>> gpurun_out/c2chk.err || exit $?
  grep '^{' gpurun_out/c2chk_one.json | python -c "import sys,json; d=json.loads(sys.stdin.read().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['diag']['unfrozen']['step_ms'])" >> gpurun_out/c2chk.txt || exit $?
done; done
