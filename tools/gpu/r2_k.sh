# GPU: GEMM + depthwise parity tests, then their micro-benchmarks.
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py -k "gemm or dw" -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/r2_k_t.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/r2_k_t.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/kbench.py copy dw_fwd gemm > gpurun_out/r2_k_b.log 2>&1
