# Round 5 (u): 32-bit / scalar index arithmetic in the BN kernels (finalize reduce, chanred, max-pool backward
# reduce, BN-backward apply, pooled / plain tails): GPU suite, in-step A/B base (HEAD) vs new (3 rounds), and a
# kernel trace of each for the per-kernel times
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
T="python -u -m pytest -p no:cacheprovider --timeout 200 --timeout-method thread -rf"
timeout -k 10 400 $T -x -q -m gpu tests > gpurun_out/u_suite.log 2>&1 || exit $?
for r in 1 2 3; do
  XCP_LIB_PATH=probe/base/libxcp.so timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 > gpurun_out/u_base_$r.log 2> gpurun_out/u_base_$r.err || exit $?
  timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 > gpurun_out/u_new_$r.log 2> gpurun_out/u_new_$r.err || exit $?
done
XCP_LIB_PATH=probe/base/libxcp.so timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/u_prof_base -o kt -- python -u bench.py --steps 5 --warmup 2 > gpurun_out/u_prof_base.log 2>&1 || exit $?
timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/u_prof_new -o kt -- python -u bench.py --steps 5 --warmup 2 > gpurun_out/u_prof_new.log 2>&1 || exit $?
