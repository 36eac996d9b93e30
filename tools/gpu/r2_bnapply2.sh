# GPU: BN-backward apply with rows per thread chosen per variant (mask 4, no mask 2): BN / tail /
# unit parity tests, kbench bnapply, headline bench.
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -v --timeout 120 --timeout-method thread -m gpu \
  -k "bn or tail or unit" > gpurun_out/ba2_tests.log 2>&1 || exit $?
timeout -k 10 120 python -u tools/kbench.py bnapply > gpurun_out/ba2_k.txt 2>&1 || exit $?
timeout -k 10 170 python -u bench.py --steps 20 --warmup 5 --cpu-baseline off --measured-peaks off \
  > gpurun_out/ba2_bench.json 2> gpurun_out/ba2_bench.err
