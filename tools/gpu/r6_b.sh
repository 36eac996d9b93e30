# Round 6 (b): full GPU suite with the two-phase NT main loop (XCP_NT_LOOP=2, gemm_nt256q_kernel) after the
# ADVICE fixes and the C5 reference-shape test; bitwise/timing A/B of the loop against the four-phase one at
# the step's shapes; the step with both loops
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
T="python -u -m pytest -p no:cacheprovider --timeout 200 --timeout-method thread -rf"
XCP_NT_LOOP=2 timeout -k 10 600 $T -x -q -m gpu tests/ --durations=15 > gpurun_out/b_gputests.log 2>&1 || exit $?
timeout -k 10 400 python -u tools/nt_loop_ab.py 3 > gpurun_out/b_ntab.log 2>&1 || exit $?
for r in 1 2; do
  timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 > gpurun_out/b_base_$r.log 2> gpurun_out/b_base_$r.err || exit $?
  XCP_NT_LOOP=2 timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 > gpurun_out/b_new_$r.log 2> gpurun_out/b_new_$r.err || exit $?
done
