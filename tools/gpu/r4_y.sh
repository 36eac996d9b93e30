# Round 4 (y): in-step A/B of the entry-flow tile rule (XCP_NT_BIG_N256=1, the default since round 3:
# outputs >= 256 wide on the 256x256 kernel from K = 128; =0: K >= 384 only), 3 interleaved rounds
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
Q="--cpu-baseline off --mode unfrozen --small-batch 0 --measured-peaks off --diag off --no-kernel-timing"
for r in 1 2 3; do
  for v in 1 0; do
    XCP_NT_BIG_N256=$v timeout -k 10 240 python bench.py $Q > gpurun_out/y_${v}_${r}.json 2>> gpurun_out/y.err || exit $?
    echo "$v $(cat gpurun_out/y_${v}_${r}.json)" >> gpurun_out/y_step.log
  done
done
