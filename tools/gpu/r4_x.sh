# Round 4 (x): weight-gradient GEMM workgroup target at HEAD (XCP_TN_TARGET_WGS: 108 / 126 (default 128
# -> 14 splits x 9 tiles) / 144 / 162 -> 12 / 14 / 16 / 18 splits at 728 x 728), 3 interleaved rounds
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
Q="--cpu-baseline off --mode unfrozen --small-batch 0 --measured-peaks off --diag off --no-kernel-timing"
for r in 1 2 3; do
  for v in 108 128 144 162; do
    XCP_TN_TARGET_WGS=$v timeout -k 10 240 python bench.py $Q > gpurun_out/x_${v}_${r}.json 2>> gpurun_out/x.err || exit $?
    echo "$v $(cat gpurun_out/x_${v}_${r}.json)" >> gpurun_out/x_step.log
  done
done
