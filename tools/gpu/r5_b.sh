# Round 5 (b): CU-partitioned backward streams (XCP_SIDE_CUS): in-step A/B, 2 interleaved rounds
#   off (default) / q=1 (64 CUs for the weight gradients, TN target 63 workgroups) / q=2 (128 CUs)
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
Q="--cpu-baseline off --mode unfrozen --small-batch 0 --measured-peaks off --diag off --no-kernel-timing"
for r in 1 2; do
  for v in off q1 q1t q2; do
    case $v in
      off) E="XCP_SIDE_CUS=0" ;;
      q1) E="XCP_SIDE_CUS=1 XCP_TN_TARGET_WGS=63" ;;
      q1t) E="XCP_SIDE_CUS=1" ;;
      q2) E="XCP_SIDE_CUS=2" ;;
    esac
    env $E timeout -k 10 240 python bench.py $Q > gpurun_out/b_${v}_${r}.json 2>> gpurun_out/b.err || exit $?
    echo "$v $(cat gpurun_out/b_${v}_${r}.json)" >> gpurun_out/b_step.log
  done
done
