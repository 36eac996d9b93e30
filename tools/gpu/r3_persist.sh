# Round 3: persistent NT kernel -- bitwise / parity tests, then the interleaved A/B.
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  -k "nt256 or persistent" > gpurun_out/r3_pt.log 2>&1 || exit $?
timeout -k 10 300 python -u tools/gemm_ab.py 5 > gpurun_out/r3_ab.log 2>&1 || exit $?
