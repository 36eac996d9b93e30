# Round 4 (zm): stem backward order at HEAD (conv1 on the matrix cores): XCP_STEM_WGRAD_EARLY=1 (default:
# conv2's weight gradient launched beside conv2's input gradient) vs 0, and XCP_STEM_BN1_FIRST, 3 rounds
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
Q="--cpu-baseline off --mode unfrozen --small-batch 0 --measured-peaks off --diag off --no-kernel-timing"
for r in 1 2 3; do
  for v in e1b1 e0b1 e1b0; do
    e=${v:1:1}; b=${v:3:1}
    XCP_STEM_WGRAD_EARLY=$e XCP_STEM_BN1_FIRST=$b timeout -k 10 240 python bench.py $Q > gpurun_out/zm_${v}_${r}.json 2>> gpurun_out/zm.err || exit $?
    echo "$v $(cat gpurun_out/zm_${v}_${r}.json)" >> gpurun_out/zm_step.log
  done
done
