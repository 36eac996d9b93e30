# Round 6 (g): the depthwise forward in the step (74.8 us) against alone (60.2 us): PMC passes on the train step and
# on the roofline ops alone -- clock (GRBM_GUI_ACTIVE), wave cycles / waits, L2 hit rate -- per dispatch
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
P="python bench.py --steps 3 --warmup 1 --cpu-baseline off --no-kernel-timing --measured-peaks off --small-batch 0 --mode unfrozen"
timeout -s KILL 240 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_BUSY_CYCLES --output-format csv -d gpurun_out/g_step_a -o p -- $P > gpurun_out/g_step_a.log 2>&1 || exit $?
timeout -s KILL 240 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d gpurun_out/g_step_b -o p -- $P > gpurun_out/g_step_b.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_BUSY_CYCLES --output-format csv -d gpurun_out/g_iso_a -o p -- python tools/kbench.py roof_ops > gpurun_out/g_iso_a.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d gpurun_out/g_iso_b -o p -- python tools/kbench.py roof_ops > gpurun_out/g_iso_b.log 2>&1 || exit $?
python tools/pmc_compare.py "dw_fwd_w2|gemm_nt256p" step=$(find gpurun_out/g_step_a -name "*counter_collection.csv" | head -1),$(find gpurun_out/g_step_b -name "*counter_collection.csv" | head -1) alone=$(find gpurun_out/g_iso_a -name "*counter_collection.csv" | head -1),$(find gpurun_out/g_iso_b -name "*counter_collection.csv" | head -1) > gpurun_out/g_compare.txt 2>&1
head -3 $(find gpurun_out/g_step_a -name "*counter_collection.csv" | head -1) > gpurun_out/g_csvhead.txt
find gpurun_out/g_step_a gpurun_out/g_step_b gpurun_out/g_iso_a gpurun_out/g_iso_b -name "*.csv" -size +4M -delete 2>/dev/null || true
