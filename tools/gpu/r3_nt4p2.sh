# Round 3: MFMA issue-rate microbenchmark, then the NT GEMM tests and A/B (epilogue row-mask change)
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 120 python -u tools/mfma_rate.py run > gpurun_out/mfma_rate2.log 2>&1 || exit $?
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -m gpu -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  -k "gemm_nt256 or persistent_bitwise or gemm_nt_stats" > gpurun_out/nt4p2_t.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/nt4p2_t.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python -u tools/gemm_ab.py 5 > gpurun_out/nt4p2_ab.log 2>&1
