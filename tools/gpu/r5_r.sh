# Round 5 (r): stem conv2 with BN1 + ReLU on load (XCP_CONV2_ACTIN) and the wgrad's asm transposed reads:
# full GPU suite, then in-step A/B: base (HEAD conv3, no act-on-load) vs new with ACTIN 0 / 1, 3 rounds
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
T="python -u -m pytest -p no:cacheprovider --timeout 200 --timeout-method thread -rf"
timeout -k 10 300 $T -x -q tests/test_gpu_kernels.py -k "conv3x3" > gpurun_out/r_conv3.log 2>&1 || exit $?
timeout -k 10 400 $T -x -q -m gpu tests > gpurun_out/r_suite.log 2>&1 || exit $?
for r in 1 2 3; do
  XCP_LIB_PATH=probe/base/libxcp.so XCP_CONV2_ACTIN=0 timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r_base_$r.log 2> gpurun_out/r_base_$r.err || exit $?
  XCP_CONV2_ACTIN=0 timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r_a0_$r.log 2> gpurun_out/r_a0_$r.err || exit $?
  XCP_CONV2_ACTIN=1 timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r_a1_$r.log 2> gpurun_out/r_a1_$r.err || exit $?
done
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/r_prof -o r -- python -u bench.py --steps 10 --warmup 3 > gpurun_out/r_prof.log 2>&1 || exit $?
