# Round 4 (ze): weight-gradient GEMM with 16 splits (XCP_TN_TARGET_WGS=144: 2 whole splits per XCD) and
# whole splits per XCD (XCP_TN_XCD_ALIGN=1) against the default (128, unaligned) and 144 unaligned; 3 rounds
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
Q="--cpu-baseline off --mode unfrozen --small-batch 0 --measured-peaks off --diag off --no-kernel-timing"
for r in 1 2 3; do
  for v in 128:0 144:1 144:0; do
    t=${v%%:*}; al=${v##*:}
    XCP_TN_TARGET_WGS=$t XCP_TN_XCD_ALIGN=$al timeout -k 10 240 python bench.py $Q > gpurun_out/ze_${t}_${al}_${r}.json 2>> gpurun_out/ze.err || exit $?
    echo "$v $(cat gpurun_out/ze_${t}_${al}_${r}.json)" >> gpurun_out/ze_step.log
  done
done
