# Round 6 (h): NT half tiles walked first (XCP_NT_HALF=1: the last round's tiles as two half tiles each, so half the
# workgroups run half a tile out of step): the bitwise tests, the op A/B, the step A/B; the depthwise forward alone
# vs right after the GEMM that writes its input
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
T="python -u -m pytest -p no:cacheprovider --timeout 200 --timeout-method thread -rf"
timeout -k 10 300 $T -x -q tests/test_gpu_kernels.py -k "half_tiles or persistent_bitwise or tile_queue or entry_flow" > gpurun_out/h_tests.log 2>&1 || exit $?
for r in 1 2 3; do
  timeout -k 10 200 python -u tools/kbench.py sparse > gpurun_out/h_sparse0_$r.log 2>&1 || exit $?
  XCP_NT_HALF=1 timeout -k 10 200 python -u tools/kbench.py sparse > gpurun_out/h_sparse1_$r.log 2>&1 || exit $?
done
for r in 1 2; do
  timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --cpu-baseline off > gpurun_out/h_base_$r.log 2> gpurun_out/h_base_$r.err || exit $?
  XCP_NT_HALF=1 timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --cpu-baseline off > gpurun_out/h_half_$r.log 2> gpurun_out/h_half_$r.err || exit $?
done
timeout -k 10 200 python -u tools/kbench.py dw_after > gpurun_out/h_dwafter.log 2>&1 || exit $?
