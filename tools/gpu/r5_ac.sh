# Round 5 (ac): the NT tile queue on the statistics-free (backward input-gradient) calls only: gemm tests,
# in-step A/B XCP_NT_DYNQ=0 / 1, 3 rounds
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
T="python -u -m pytest -p no:cacheprovider --timeout 200 --timeout-method thread -rf"
timeout -k 10 300 $T -x -q tests/test_gpu_kernels.py -k "gemm or nt" > gpurun_out/ac_tests.log 2>&1 || exit $?
for r in 1 2 3; do
  XCP_NT_DYNQ=0 timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 > gpurun_out/ac_off_$r.log 2> gpurun_out/ac_off_$r.err || exit $?
  XCP_NT_DYNQ=1 timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 > gpurun_out/ac_on_$r.log 2> gpurun_out/ac_on_$r.err || exit $?
done
