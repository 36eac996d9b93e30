# Round 6 (v6): record of HEAD (v5 + the NT last K-tile half skip) on one box: full -m gpu suite, smoke, default bench line, kernel trace +
# per-stream timeline + per-role summary of the headline step, HBM traffic per launch (step and op PMC passes);
# round 6 defaults: weight-gradient loop gemm_tn256q, persistent LSTM forward, non-temporal NT C stores, the fused
# block1 forward's width gate, the C4 one-graph replay, the clip-grouped LSTM backward default (small B); + the C4 / C5 / C2 lines, the depthwise in-step
# PMC comparison (tools/pmc_compare.py) and the DDP proxy line
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
( while true; do date >> gpurun_out/v6_heartbeat.txt; sleep 50; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
timeout -k 10 1100 python -u -m pytest tests -m gpu -v -p no:cacheprovider --timeout 500 --timeout-method thread -rf --durations=15 > gpurun_out/v6_suite.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/v6_suite.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/v6_smoke.log 2>&1 || exit $?
timeout -k 10 600 python bench.py > gpurun_out/v6_bench.json 2> gpurun_out/v6_bench.err || exit $?
B="python bench.py --cpu-baseline off --mode unfrozen --steps 5 --warmup 2 --small-batch 0 --measured-peaks off --diag off"
XCP_BENCH_OP_ORDER=gpurun_out/v6_oporder.json timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_r6v6 -o kt -- $B > gpurun_out/v6_prof.log 2>&1 || exit $?
python tools/stream_timeline.py "$(find gpurun_out/prof_r6v6 -name "*kernel_trace.csv" | head -1)" 40 > gpurun_out/v6_timeline.txt 2>&1
python tools/prof_summary.py gpurun_out/prof_r6v6 60 --op-order gpurun_out/v6_oporder.json > gpurun_out/v6_kernels.txt 2>&1
P="python bench.py --cpu-baseline off --mode unfrozen --steps 3 --warmup 1 --small-batch 0 --measured-peaks off --diag off --no-kernel-timing"
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/v6_pmct_fetch -o p -- $P > gpurun_out/v6_pmct_f.log 2>&1 || exit $?
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/v6_pmct_write -o p -- $P > gpurun_out/v6_pmct_w.log 2>&1 || exit $?
python tools/pmc_traffic.py $(find gpurun_out/v6_pmct_fetch -name "*counter_collection.csv" | head -1) $(find gpurun_out/v6_pmct_write -name "*counter_collection.csv" | head -1) gpurun_out/v6_step_traffic.json > gpurun_out/v6_pmct.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/v6_pmco_fetch -o p -- python tools/kbench.py roof_ops > gpurun_out/v6_pmco_f.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/v6_pmco_write -o p -- python tools/kbench.py roof_ops > gpurun_out/v6_pmco_w.log 2>&1 || exit $?
python tools/pmc_traffic.py $(find gpurun_out/v6_pmco_fetch -name "*counter_collection.csv" | head -1) $(find gpurun_out/v6_pmco_write -name "*counter_collection.csv" | head -1) gpurun_out/v6_optraffic.json > gpurun_out/v6_pmco.log 2>&1
G="python bench.py --gpus 2 --cpu-baseline off --mode unfrozen --steps 3 --warmup 1 --small-batch 0 --measured-peaks off --diag off --no-kernel-timing"
XCP_BENCH_BACKEND=gloo timeout -k 10 400 $G > gpurun_out/v6_2rank_gloo.json 2> gpurun_out/v6_2rank_gloo.err || exit $?
# keep the merged-back output small: the summaries above are what is kept
find gpurun_out/prof_r6v6 gpurun_out/v6_pmct_fetch gpurun_out/v6_pmct_write gpurun_out/v6_pmco_fetch gpurun_out/v6_pmco_write -name "*.csv" -size +2M -delete 2>/dev/null || true
timeout -k 10 300 python -u bench.py --model lstma --cpu-baseline off > gpurun_out/v6_lstma.json 2> gpurun_out/v6_lstma.err || exit $?
P2="python bench.py --steps 3 --warmup 1 --cpu-baseline off --no-kernel-timing --measured-peaks off --small-batch 0 --mode unfrozen"
timeout -s KILL 240 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_BUSY_CYCLES --output-format csv -d gpurun_out/v6_gstep_a -o p -- $P2 > gpurun_out/v6_gstep_a.log 2>&1 || exit $?
timeout -s KILL 240 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d gpurun_out/v6_gstep_b -o p -- $P2 > gpurun_out/v6_gstep_b.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_BUSY_CYCLES --output-format csv -d gpurun_out/v6_giso_a -o p -- python tools/kbench.py roof_ops > gpurun_out/v6_giso_a.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d gpurun_out/v6_giso_b -o p -- python tools/kbench.py roof_ops > gpurun_out/v6_giso_b.log 2>&1 || exit $?
head -3 $(find gpurun_out/v6_gstep_a -name "*counter_collection.csv" | head -1) > gpurun_out/v6_csvhead.txt
python tools/pmc_compare.py "dw_fwd_w2|gemm_nt256p|dw_bwd_lds" step=$(find gpurun_out/v6_gstep_a -name "*counter_collection.csv" | head -1),$(find gpurun_out/v6_gstep_b -name "*counter_collection.csv" | head -1) alone=$(find gpurun_out/v6_giso_a -name "*counter_collection.csv" | head -1),$(find gpurun_out/v6_giso_b -name "*counter_collection.csv" | head -1) > gpurun_out/v6_dwpmc.txt 2>&1
timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --cpu-baseline off --ddp-proxy 8 > gpurun_out/v6_proxy.json 2> gpurun_out/v6_proxy.err || exit $?
find gpurun_out/v6_gstep_a gpurun_out/v6_gstep_b gpurun_out/v6_giso_a gpurun_out/v6_giso_b -name "*.csv" -size +3M -delete 2>/dev/null || true
timeout -k 10 300 python -u bench.py --model auface --cpu-baseline off > gpurun_out/v6_auface.json 2> gpurun_out/v6_auface.err || exit $?
timeout -k 10 300 python -u bench.py --model xception --cpu-baseline off > gpurun_out/v6_xception.json 2> gpurun_out/v6_xception.err || exit $?
