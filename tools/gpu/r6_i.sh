# Round 6 (i): persistent LSTM backward with the reader-coalesced dh-partial layout: LSTM tests, fwd/bwd A/B, the C4
# line with the default (persistent forward, per-step backward) and with both persistent
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
T="python -u -m pytest -p no:cacheprovider --timeout 200 --timeout-method thread -rf"
timeout -k 10 300 $T -x -q tests/test_gpu_kernels.py -k "lstm" > gpurun_out/i_lstmtests.log 2>&1 || exit $?
timeout -k 10 300 python -u tools/lstm_ab.py 3 > gpurun_out/i_lstmab.log 2>&1 || exit $?
for r in 1 2; do
  timeout -k 10 200 python -u bench.py --model lstma --steps 20 --warmup 5 --cpu-baseline off > gpurun_out/i_ldef_$r.log 2> gpurun_out/i_ldef_$r.err || exit $?
  XCP_LSTM_PERSIST=1 timeout -k 10 200 python -u bench.py --model lstma --steps 20 --warmup 5 --cpu-baseline off > gpurun_out/i_lboth_$r.log 2> gpurun_out/i_lboth_$r.err || exit $?
  XCP_LSTM_PERSIST=0 timeout -k 10 200 python -u bench.py --model lstma --steps 20 --warmup 5 --cpu-baseline off > gpurun_out/i_lnone_$r.log 2> gpurun_out/i_lnone_$r.err || exit $?
done
# (j) the pointwise GEMM's C stores with sc1 (write-through, not kept in L2) or nt, against plain: the GEMM alone, the
# depthwise forward right after it, the step
for r in 1 2; do
  timeout -k 10 200 python -u tools/kbench.py dw_after ntprobe > gpurun_out/j_base_$r.log 2>&1 || exit $?
  XCP_LIB_PATH=probe/csc1/libxcp.so timeout -k 10 200 python -u tools/kbench.py dw_after ntprobe > gpurun_out/j_sc1_$r.log 2>&1 || exit $?
  XCP_LIB_PATH=probe/cnt/libxcp.so timeout -k 10 200 python -u tools/kbench.py dw_after ntprobe > gpurun_out/j_nt_$r.log 2>&1 || exit $?
done
for r in 1 2; do
  timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --cpu-baseline off > gpurun_out/j_sbase_$r.log 2> gpurun_out/j_sbase_$r.err || exit $?
  XCP_LIB_PATH=probe/csc1/libxcp.so timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --cpu-baseline off > gpurun_out/j_ssc1_$r.log 2> gpurun_out/j_ssc1_$r.err || exit $?
  XCP_LIB_PATH=probe/cnt/libxcp.so timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --cpu-baseline off > gpurun_out/j_snt_$r.log 2> gpurun_out/j_snt_$r.err || exit $?
done
