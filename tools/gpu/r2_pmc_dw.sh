# GPU: PMC passes on the isolated middle-flow depthwise kernels.
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for k in dwf_only dwb_only; do
  timeout -s KILL 120 rocprofv3 --pmc TA_TA_BUSY TA_ADDR_STALLED_BY_TC_CYCLES GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/pmc_ta_$k -o p -- python tools/kbench.py $k > gpurun_out/pmc_ta_$k.log 2>&1 || exit $?
  timeout -s KILL 120 rocprofv3 --pmc TCP_TCC_READ_REQ_LATENCY TCP_TCC_READ_REQ TCP_PENDING_STALL_CYCLES TCP_TCR_TCP_STALL_CYCLES --output-format csv -d gpurun_out/pmc_tcp_$k -o p -- python tools/kbench.py $k > gpurun_out/pmc_tcp_$k.log 2>&1 || exit $?
  timeout -s KILL 120 rocprofv3 --pmc TCC_HIT TCC_MISS TD_TD_BUSY TD_TC_STALL --output-format csv -d gpurun_out/pmc_tcc_$k -o p -- python tools/kbench.py $k > gpurun_out/pmc_tcc_$k.log 2>&1 || exit $?
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_INSTS_VMEM SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_WAIT_INST_ANY --output-format csv -d gpurun_out/pmc_sq_$k -o p -- python tools/kbench.py $k > gpurun_out/pmc_sq_$k.log 2>&1 || exit $?
done
echo ok
