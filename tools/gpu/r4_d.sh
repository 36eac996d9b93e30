# Round 4 (d): the 2-rank gloo path (ranks share cuda:0) with the communication stream vs the
# round-3 launch order, at 4 and 16 clips/rank; the suite's new kernel tests
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest -p no:cacheprovider --timeout 300 --timeout-method thread -rf tests/test_gpu_kernels.py -q -k "row_bands or permute_batch" > gpurun_out/d_tests.log 2>&1 || exit $?
S="--steps 3 --warmup 2 --mode unfrozen --cpu-baseline off --small-batch 0 --measured-peaks off --no-kernel-timing --diag off"
for v in 1 0; do
  XCP_DDP_COMM_STREAM=$v XCP_BENCH_BACKEND=gloo timeout -k 10 300 python bench.py --gpus 2 --batch 4 $S > gpurun_out/d_g2_b4_c$v.json 2> gpurun_out/d_g2_b4_c$v.err || exit $?
done
for v in 1 0; do
  XCP_DDP_COMM_STREAM=$v XCP_BENCH_BACKEND=gloo timeout -k 10 300 python bench.py --gpus 2 $S > gpurun_out/d_g2_b16_c$v.json 2> gpurun_out/d_g2_b16_c$v.err || exit $?
done
timeout -k 10 200 python bench.py --cpu-baseline off --small-batch 0 --measured-peaks off --diag off > gpurun_out/d_b.json 2> gpurun_out/d_b.err || exit $?
