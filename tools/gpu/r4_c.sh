# Round 4 (c): depthwise backward row bands (kernel times, in-step A/B), the 2-rank gloo path at 4
# clips/rank against world 1 at 4 clips (ranks share cuda:0: gloo, not RCCL)
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u tools/dw_bands.py > gpurun_out/c_bands.log 2>&1 || exit $?
Q="--cpu-baseline off --mode unfrozen --small-batch 0 --measured-peaks off --diag off --no-kernel-timing"
for v in 1x0 2x0 1x1 2x1 1x0 2x0 1x1 2x1; do
  XCP_DW_BWD_BANDS=${v%x*} XCP_DW_BWD_XCD=${v#*x} timeout -k 10 200 python bench.py $Q > gpurun_out/c_step_dw$v.json 2>> gpurun_out/c_step_dw.err || exit $?
  echo "$v $(cat gpurun_out/c_step_dw$v.json)" >> gpurun_out/c_step_dw.log
done
S="--steps 4 --warmup 2 --batch 4 --mode unfrozen --cpu-baseline off --small-batch 0 --measured-peaks off --no-kernel-timing"
XCP_BENCH_BACKEND=gloo timeout -k 10 300 python bench.py --gpus 2 $S > gpurun_out/c_g2.json 2> gpurun_out/c_g2.err || exit $?
timeout -k 10 300 python bench.py $S > gpurun_out/c_g1.json 2> gpurun_out/c_g1.err || exit $?
# weight-gradient split layout in the step: XCD-whole splits (S a multiple of 8) at targets 72 / 144 vs default
Q="--cpu-baseline off --mode unfrozen --small-batch 0 --measured-peaks off --diag off --no-kernel-timing"
for v in base xcd72 xcd144 base xcd72 xcd144; do
  case $v in base) E="";; xcd72) E="XCP_TN_XCD_SPLITS=1 XCP_TN_TARGET_WGS=72";; xcd144) E="XCP_TN_XCD_SPLITS=1 XCP_TN_TARGET_WGS=144";; esac
  env $E timeout -k 10 200 python bench.py $Q > gpurun_out/c_tn_$v.json 2>> gpurun_out/c_tn.err || exit $?
  echo "$v $(cat gpurun_out/c_tn_$v.json)" >> gpurun_out/c_tn.log
done
