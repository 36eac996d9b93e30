# Round 5 (ah): queued (statistics-free) NT calls keep every row on the persistent kernel (default) vs the
# sparse last round on the 128x128 kernel (XCP_NT_SPARSE_DGRAD=1): gemm tests, in-step A/B, 3 rounds
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest -p no:cacheprovider --timeout 200 --timeout-method thread -rf -x -q tests/test_gpu_kernels.py -k "gemm" > gpurun_out/ah_tests.log 2>&1 || exit $?
for r in 1 2 3; do
  XCP_NT_SPARSE_DGRAD=1 timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 > gpurun_out/ah_old_$r.log 2> gpurun_out/ah_old_$r.err || exit $?
  timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 > gpurun_out/ah_new_$r.log 2> gpurun_out/ah_new_$r.err || exit $?
done
