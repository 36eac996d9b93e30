# Round 4 (zk): per-kernel effective clock and MFMA-busy fraction of the headline step at HEAD
# (GRBM_GUI_ACTIVE and SQ_VALU_MFMA_BUSY_CYCLES, separate --pmc passes; tools/eff_clock.py)
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
P="python bench.py --cpu-baseline off --mode unfrozen --steps 3 --warmup 1 --small-batch 0 --measured-peaks off --diag off --no-kernel-timing"
timeout -s KILL 240 rocprofv3 --pmc GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/zk_grbm -o p -- $P > gpurun_out/zk_g.log 2>&1 || exit $?
timeout -s KILL 240 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES --output-format csv -d gpurun_out/zk_sq -o p -- $P > gpurun_out/zk_s.log 2>&1 || exit $?
python tools/eff_clock.py $(find gpurun_out/zk_grbm -name "*counter_collection.csv" | head -1) $(find gpurun_out/zk_sq -name "*counter_collection.csv" | head -1) > gpurun_out/zk_clock_mfma.txt 2>&1
