# Round 5 (x): fused unit backward with the 2 GB num_records and explicit out-of-range offsets (vs the exact
# split span of r5_w): unit tests, kbench unitbwd base (HEAD) / new, two rounds
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
T="python -u -m pytest -p no:cacheprovider --timeout 200 --timeout-method thread -rf"
timeout -k 10 300 $T -x -q tests/test_gpu_kernels.py tests/test_gpu_modules.py -k "unit" > gpurun_out/x_tests.log 2>&1 || exit $?
for r in 1 2; do
  XCP_LIB_PATH=probe/base/libxcp.so timeout -k 10 200 python -u tools/kbench.py unitbwd > gpurun_out/x_ub_base_$r.log 2>&1 || exit $?
  timeout -k 10 200 python -u tools/kbench.py unitbwd > gpurun_out/x_ub_new_$r.log 2>&1 || exit $?
done
