# Round 5 (q): fused block1 forward, Y staged through LDS for 16-B row stores (probe/y1) vs shipped
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
T="python -u -m pytest -p no:cacheprovider --timeout 200 --timeout-method thread -rf"
XCP_LIB_PATH=probe/y1/libxcp.so timeout -k 10 300 $T -x -q tests/test_gpu_kernels.py -k "sep_fwd" > gpurun_out/q_tests.log 2>&1 || exit $?
for r in 1 2; do
  timeout -k 10 200 python -u tools/sep_bench.py 10 > gpurun_out/q_base_$r.log 2>&1 || exit $?
  XCP_LIB_PATH=probe/y1/libxcp.so timeout -k 10 200 python -u tools/sep_bench.py 10 > gpurun_out/q_y1_$r.log 2>&1 || exit $?
done
