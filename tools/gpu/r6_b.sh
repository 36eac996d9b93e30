# Round 6 (b): the two-phase NT main loop (gemm_nt256q_kernel): GEMM tests, bitwise/timing A/B against
# the four-phase loop at the step's shapes, then the step with both loops
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
T="python -u -m pytest -p no:cacheprovider --timeout 200 --timeout-method thread -rf"
timeout -k 10 300 $T -x -q -m gpu tests/test_gpu_kernels.py -k "gemm or nt" > gpurun_out/b_gemmtests.log 2>&1 || exit $?
timeout -k 10 400 python -u tools/nt_loop_ab.py 3 > gpurun_out/b_ntab.log 2>&1 || exit $?
for r in 1 2; do
  timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 > gpurun_out/b_base_$r.log 2> gpurun_out/b_base_$r.err || exit $?
  XCP_NT_LOOP=2 timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 > gpurun_out/b_new_$r.log 2> gpurun_out/b_new_$r.err || exit $?
done
