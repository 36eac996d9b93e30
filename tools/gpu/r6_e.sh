# Round 6 (e + f): persistent LSTM with every load of a step issued before its first use (512-register waves,
# compile-time reduce-scatter): LSTM tests, fwd/bwd A/B, the lstma step A/B; the weight-gradient loop
# (XCP_TN_LOOP=2) in the lstmv step with the default NT loop
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
T="python -u -m pytest -p no:cacheprovider --timeout 200 --timeout-method thread -rf"
timeout -k 10 300 $T -x -q tests/test_gpu_kernels.py -k "lstm" > gpurun_out/e_lstmtests.log 2>&1 || exit $?
timeout -k 10 300 python -u tools/lstm_ab.py 3 > gpurun_out/e_lstmab.log 2>&1 || exit $?
for r in 1 2; do
  XCP_LSTM_PERSIST=0 timeout -k 10 200 python -u bench.py --model lstma --steps 20 --warmup 5 --cpu-baseline off > gpurun_out/e_lstep_$r.log 2> gpurun_out/e_lstep_$r.err || exit $?
  XCP_LSTM_PERSIST=1 timeout -k 10 200 python -u bench.py --model lstma --steps 20 --warmup 5 --cpu-baseline off > gpurun_out/e_lpers_$r.log 2> gpurun_out/e_lpers_$r.err || exit $?
done
for r in 1 2; do
  timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --cpu-baseline off > gpurun_out/e_base_$r.log 2> gpurun_out/e_base_$r.err || exit $?
  XCP_TN_LOOP=2 timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --cpu-baseline off > gpurun_out/e_tn2_$r.log 2> gpurun_out/e_tn2_$r.err || exit $?
done
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for r in 1 2; do
  timeout -k 10 200 python -u tools/kbench.py ntprobe > gpurun_out/f_base_$r.log 2>&1 || exit $?
  XCP_LIB_PATH=probe/oobstore/libxcp.so timeout -k 10 200 python -u tools/kbench.py ntprobe > gpurun_out/f_oob_$r.log 2>&1 || exit $?
  XCP_LIB_PATH=probe/nostore/libxcp.so timeout -k 10 200 python -u tools/kbench.py ntprobe > gpurun_out/f_nost_$r.log 2>&1 || exit $?
done
