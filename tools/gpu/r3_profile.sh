# Round 3 HEAD profiles: rocprofv3 kernel trace + stats of the bench (unfrozen headline step),
# FETCH_SIZE / WRITE_SIZE passes (HBM traffic per launch), GRBM_GUI_ACTIVE (effective clock per
# dispatch) and an SQ pass (MFMA busy, waits) -- each counter set in its own run.
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
B="python bench.py --cpu-baseline off --mode unfrozen --steps 5 --warmup 2 --small-batch 0 --measured-peaks off --diag off"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_r3 -o kt -- $B > gpurun_out/r3_prof.log 2>&1 || exit $?
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc3_fetch -o p -- $B --no-kernel-timing > gpurun_out/r3_pmc_f.log 2>&1 || exit $?
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc3_write -o p -- $B --no-kernel-timing > gpurun_out/r3_pmc_w.log 2>&1 || exit $?
timeout -s KILL 240 rocprofv3 --pmc GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/pmc3_grbm -o p -- $B --no-kernel-timing > gpurun_out/r3_pmc_g.log 2>&1 || exit $?
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VMEM --output-format csv -d gpurun_out/pmc3_sq -o p -- $B --no-kernel-timing > gpurun_out/r3_pmc_sq.log 2>&1 || exit $?
echo ok
