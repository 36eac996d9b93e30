# Round 4 (e): persistent depthwise forward (bitwise tests, kernel A/B, in-step A/B with the
# XCD-ordered depthwise backward)
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest -p no:cacheprovider --timeout 300 --timeout-method thread -rf tests/test_gpu_kernels.py -q -k "persistent_bitwise or row_bands or permute_batch or dw_fwd_bwd" > gpurun_out/e_tests.log 2>&1 || exit $?
timeout -k 10 300 python -u tools/dw_fwd_ab.py > gpurun_out/e_fwd_ab.log 2>&1 || exit $?
Q="--cpu-baseline off --mode unfrozen --small-batch 0 --measured-peaks off --diag off --no-kernel-timing"
for v in 0 2 4 0 2 4; do
  XCP_DW_BWD_XCD=1 XCP_DW_FWD_P=$v timeout -k 10 200 python bench.py $Q > gpurun_out/e_step_p$v.json 2>> gpurun_out/e_step.err || exit $?
  echo "$v $(cat gpurun_out/e_step_p$v.json)" >> gpurun_out/e_step.log
done
# the 2-rank gloo path (ranks share cuda:0): collectives launched from the side stream (default),
# the main stream (round 3) or a communication stream
S="--steps 3 --warmup 2 --batch 4 --mode unfrozen --cpu-baseline off --small-batch 0 --measured-peaks off --no-kernel-timing --diag off"
for v in side main comm; do
  XCP_DDP_LAUNCH=$v XCP_BENCH_BACKEND=gloo timeout -k 10 300 python bench.py --gpus 2 $S > gpurun_out/e_g2_$v.json 2> gpurun_out/e_g2_$v.err || exit $?
done
timeout -k 10 300 python -u -m pytest -p no:cacheprovider --timeout 300 --timeout-method thread -rf tests/test_gpu_ddp.py -q > gpurun_out/e_ddp_tests.log 2>&1 || exit $?
