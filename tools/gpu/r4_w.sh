# Round 4 (w): in-step A/B of the middle flow's channel pitch, 736 (default) against 768 (whole 128-B
# lines per pixel row: r02's isolated GEMMs 3-5 % and depthwise backward 5 % faster, depthwise forward
# 9 % slower, +4.3 % bytes) -- XCP_PAD_728, 3 interleaved rounds
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
Q="--cpu-baseline off --mode unfrozen --small-batch 0 --measured-peaks off --diag off --no-kernel-timing"
for r in 1 2 3; do
  for v in 736 768; do
    XCP_PAD_728=$v timeout -k 10 240 python bench.py $Q > gpurun_out/w_${v}_${r}.json 2>> gpurun_out/w.err || exit $?
    echo "$v $(cat gpurun_out/w_${v}_${r}.json)" >> gpurun_out/w_step.log
  done
done
XCP_PAD_728=768 timeout -k 10 200 python -u tools/kbench.py roof_ops > gpurun_out/w_kb768.log 2>&1 || exit $?
timeout -k 10 200 python -u tools/kbench.py roof_ops > gpurun_out/w_kb736.log 2>&1 || exit $?
