# Round 4 (b): full -m gpu suite at HEAD, HEAD bench (default line), kernel trace + per-stream
# timeline of the headline step, in-step ablation
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread -rf --durations=15 > gpurun_out/b_suite.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/b_suite.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 600 python bench.py > gpurun_out/b_b.json 2> gpurun_out/b_b.err || exit $?
B="python bench.py --cpu-baseline off --mode unfrozen --steps 5 --warmup 2 --small-batch 0 --measured-peaks off --diag off"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_r4b -o kt -- $B > gpurun_out/b_prof.log 2>&1 || exit $?
python tools/stream_timeline.py "$(find gpurun_out/prof_r4b -name "*kernel_trace.csv" | head -1)" 40 > gpurun_out/b_timeline.txt 2>&1
python tools/prof_summary.py gpurun_out/prof_r4b 60 > gpurun_out/b_kernels.txt 2>&1
timeout -k 10 300 python -u tools/step_ablation.py --rounds 3 gemm_tn gemm_nt:728fwd gemm_nt:728dgrad gemm_nt:dgrad gemm_nt:fwd dw_bwd dw_fwd bn_bwd_apply colreduce_multi bn_bwd_reduce unit_bwd bn_finalize_part+bn_bwd_finalize_part maxpool_bwd_bnred > gpurun_out/b_ablation.log 2>&1
