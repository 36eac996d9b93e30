# Round 4 (b): HEAD bench (default line), the 2-rank gloo path at 4 clips/rank against world 1 at
# 4 clips (ranks share cuda:0: gloo, not RCCL), kernel trace + per-stream timeline of the headline step
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python bench.py > gpurun_out/b_b.json 2> gpurun_out/b_b.err || exit $?
S="--steps 4 --warmup 2 --batch 4 --mode unfrozen --cpu-baseline off --small-batch 0 --measured-peaks off --no-kernel-timing"
XCP_BENCH_BACKEND=gloo timeout -k 10 300 python bench.py --gpus 2 $S > gpurun_out/b_g2.json 2> gpurun_out/b_g2.err || exit $?
timeout -k 10 300 python bench.py $S > gpurun_out/b_g1.json 2> gpurun_out/b_g1.err || exit $?
B="python bench.py --cpu-baseline off --mode unfrozen --steps 5 --warmup 2 --small-batch 0 --measured-peaks off --diag off"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_r4b -o kt -- $B > gpurun_out/b_prof.log 2>&1 || exit $?
python tools/stream_timeline.py "$(find gpurun_out/prof_r4b -name "*kernel_trace.csv" | head -1)" 40 > gpurun_out/b_timeline.txt 2>&1
python tools/prof_summary.py gpurun_out/prof_r4b 60 > gpurun_out/b_kernels.txt 2>&1

timeout -k 10 300 python -u tools/step_ablation.py --rounds 3 gemm_tn gemm_nt:728fwd gemm_nt:728dgrad gemm_nt:dgrad gemm_nt:fwd dw_bwd dw_fwd bn_bwd_apply colreduce_multi bn_bwd_reduce unit_bwd bn_finalize_part+bn_bwd_finalize_part maxpool_bwd_bnred > gpurun_out/b_ablation.log 2>&1
