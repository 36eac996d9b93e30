# Round 3: NT phase stamps + persistent A/B (interleaved).
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 200 python -u tools/gemm_phase.py run > gpurun_out/r3_phase.log 2>&1 || exit $?
timeout -k 10 300 python -u tools/gemm_ab.py 5 > gpurun_out/r3_ab2.log 2>&1 || exit $?
