# Round 6 (d): new kernels first, each in its own step -- persistent H = 512 LSTM recurrence (tests_lstm), the
# two-phase NT loop (XCP_NT_LOOP=2) GEMM tests; then the full GPU suite with both; NT loop A/B at the step's
# shapes; the lstmv step with both NT loops; the lstma step with per-step / persistent LSTM kernels; the DDP
# proxy (8-rank RCCL stand-in) on the lstmv step
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
T="python -u -m pytest -p no:cacheprovider --timeout 200 --timeout-method thread -rf"
timeout -k 10 300 $T -x -q tests/test_gpu_kernels.py -k "lstm" > gpurun_out/d_lstmtests.log 2>&1 || exit $?
XCP_NT_LOOP=2 timeout -k 10 300 $T -x -q tests/test_gpu_kernels.py -k "gemm or nt" > gpurun_out/d_nttests.log 2>&1 || exit $?
XCP_LSTM_PERSIST=1 XCP_NT_LOOP=2 timeout -k 10 600 $T -x -q -m gpu tests/ --durations=15 > gpurun_out/d_gputests.log 2>&1 || exit $?
timeout -k 10 400 python -u tools/nt_loop_ab.py 3 > gpurun_out/d_ntab.log 2>&1 || exit $?
for r in 1 2; do
  timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --cpu-baseline off > gpurun_out/d_base_$r.log 2> gpurun_out/d_base_$r.err || exit $?
  XCP_NT_LOOP=2 timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --cpu-baseline off > gpurun_out/d_new_$r.log 2> gpurun_out/d_new_$r.err || exit $?
done
for r in 1 2; do
  XCP_LSTM_PERSIST=0 timeout -k 10 200 python -u bench.py --model lstma --steps 20 --warmup 5 --cpu-baseline off > gpurun_out/d_lstep_$r.log 2> gpurun_out/d_lstep_$r.err || exit $?
  XCP_LSTM_PERSIST=1 timeout -k 10 200 python -u bench.py --model lstma --steps 20 --warmup 5 --cpu-baseline off > gpurun_out/d_lpers_$r.log 2> gpurun_out/d_lpers_$r.err || exit $?
done
timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --cpu-baseline off --ddp-proxy 8 > gpurun_out/d_proxy.log 2> gpurun_out/d_proxy.err || exit $?
timeout -k 10 300 $T -x -q tests/test_gpu_kernels.py -k "gemm_tn" > gpurun_out/d_tntests.log 2>&1 || exit $?
timeout -k 10 400 python -u tools/tn_loop_ab.py 3 > gpurun_out/d_tnab.log 2>&1 || exit $?
for r in 1 2; do
  XCP_NT_LOOP=2 XCP_TN_LOOP=2 timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --cpu-baseline off > gpurun_out/d_tn2_$r.log 2> gpurun_out/d_tn2_$r.err || exit $?
done
