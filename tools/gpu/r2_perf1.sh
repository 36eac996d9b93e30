# GPU: failing-test re-run, kernel micro-benchmarks (incl. hipBLASLt on the same GEMM shapes),
# and a kernel-trace profile of the bench with the weight-gradient side stream off (isolated
# kernel durations) and on.
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u -m pytest tests/test_gpu_modules.py tests/test_gpu_train_step.py -q --timeout 300 --timeout-method thread -rf -p no:cacheprovider > gpurun_out/r2_t3.log 2>&1
echo "pytest rc=$?" >> gpurun_out/r2_t3.log
timeout -k 10 300 python -u tools/kbench.py copy dw_fwd dw_bwd gemm bn blas cold > gpurun_out/r2_kbench.log 2>&1 || exit $?
XCP_WGRAD_STREAM=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_ws0 -o kt -- python bench.py --cpu-baseline off --mode unfrozen --steps 5 --warmup 2 > gpurun_out/r2_prof_ws0.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_ws1 -o kt -- python bench.py --cpu-baseline off --mode unfrozen --steps 5 --warmup 2 > gpurun_out/r2_prof_ws1.log 2>&1
