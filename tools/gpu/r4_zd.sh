# Round 4 (zd): the persistent NT kernel's sparse last round: op times at every persistent shape of the step
# (tile 0 auto vs tile 3 every row persistent, tools/kbench.py sparse) and the step with XCP_NT_SPARSE=0 / 1
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u tools/kbench.py sparse > gpurun_out/zd_kb.log 2>&1 || exit $?
Q="--cpu-baseline off --mode unfrozen --small-batch 0 --measured-peaks off --diag off --no-kernel-timing"
for r in 1 2 3; do
  for v in 1 0; do
    XCP_NT_SPARSE=$v timeout -k 10 240 python bench.py $Q > gpurun_out/zd_${v}_${r}.json 2>> gpurun_out/zd.err || exit $?
    echo "$v $(cat gpurun_out/zd_${v}_${r}.json)" >> gpurun_out/zd_step.log
  done
done
