# Round 5 (d): pipelined depthwise forward ring shapes (XCP_DW_FWD_PIPE=1..4) against the one-tile kernel:
# bitwise test, then kernel timings at the step's shapes
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
T="python -u -m pytest -p no:cacheprovider --timeout 150 --timeout-method thread -rf"
timeout -k 10 300 $T -q tests/test_gpu_kernels.py -k "dw_fwd_pipelined" > gpurun_out/d_tests.log 2>&1 || exit $?
for v in 0 1 2 3 4; do XCP_DW_FWD_PIPE=$v timeout -k 10 200 python tools/kbench.py dwshapes > gpurun_out/d_kb_$v.log 2>&1 || exit $?; done
