# Round 5 (aa): fused Adam on 16-B vectors: optimizer tests, kernel trace of base / new (opt_adam time),
# in-step A/B base (HEAD) vs new, 3 rounds
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
T="python -u -m pytest -p no:cacheprovider --timeout 200 --timeout-method thread -rf"
timeout -k 10 300 $T -x -q tests/test_gpu_kernels.py tests/test_gpu_train_step.py tests/test_gpu_model.py -k "adam or optim" > gpurun_out/aa_tests.log 2>&1 || exit $?
XCP_LIB_PATH=probe/base/libxcp.so timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/aa_prof_base -o kt -- python -u bench.py --steps 5 --warmup 2 > gpurun_out/aa_prof_base.log 2>&1 || exit $?
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/aa_prof_new -o kt -- python -u bench.py --steps 5 --warmup 2 > gpurun_out/aa_prof_new.log 2>&1 || exit $?
find gpurun_out/aa_prof_base gpurun_out/aa_prof_new -name "*kernel_trace.csv" -delete
for r in 1 2 3; do
  XCP_LIB_PATH=probe/base/libxcp.so timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 > gpurun_out/aa_base_$r.log 2> gpurun_out/aa_base_$r.err || exit $?
  timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 > gpurun_out/aa_new_$r.log 2> gpurun_out/aa_new_$r.err || exit $?
done
