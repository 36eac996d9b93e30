# GPU: GEMM parity tests (incl. the >2 GB global-address path), then the ablation timings.
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -k "gemm" -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/r2_gemm_t.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/r2_gemm_t.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/gemm_exp.py run > gpurun_out/r2_exp.log 2>&1
