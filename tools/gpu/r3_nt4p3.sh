# Round 3: 4-wave persistent NT kernel phase stamps (variants), then the NT GEMM tests and A/B
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 150 python -u tools/gemm_stamps4.py run > gpurun_out/stamps4p.log 2>&1 || exit $?
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -m gpu -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  -k "gemm_nt256 or persistent_bitwise or gemm_nt_stats" > gpurun_out/nt4p3_t.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/nt4p3_t.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python -u tools/gemm_ab.py 5 > gpurun_out/nt4p3_ab.log 2>&1
