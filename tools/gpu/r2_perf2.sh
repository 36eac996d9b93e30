# GPU: GEMM fixed-cost / main-loop sweep and PMC passes (MFMA busy, LDS, HBM traffic) on the
# middle-flow pointwise GEMMs in isolation.
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 python -u tools/kbench.py ksweep gemm > gpurun_out/r2_ksweep.log 2>&1 || exit $?
SQ=SQ_VALU_MFMA_BUSY_CYCLES,SQ_BUSY_CYCLES,SQ_WAVE_CYCLES,SQ_LDS_BANK_CONFLICT,SQ_LDS_IDX_ACTIVE,SQ_WAIT_INST_LDS,GRBM_GUI_ACTIVE
for k in nt_only tn_only; do
  timeout -s KILL 120 rocprofv3 --pmc $SQ --output-format csv -d gpurun_out/pmc_sq_$k -o p -- python tools/kbench.py $k > gpurun_out/pmc_sq_$k.log 2>&1 || exit $?
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_f_$k -o p -- python tools/kbench.py $k > gpurun_out/pmc_f_$k.log 2>&1 || exit $?
  timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_w_$k -o p -- python tools/kbench.py $k > gpurun_out/pmc_w_$k.log 2>&1 || exit $?
done
echo done
