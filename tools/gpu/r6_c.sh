# Round 6 (c): persistent H = 512 LSTM recurrence (one launch per direction): LSTM kernel tests, the
# XceptionLSTMA model tests, the C4 line with the per-step kernels (XCP_LSTM_PERSIST=0) and the persistent ones
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
T="python -u -m pytest -p no:cacheprovider --timeout 200 --timeout-method thread -rf"
timeout -k 10 300 $T -x -q tests/test_gpu_kernels.py -k "lstm" > gpurun_out/c_lstmtests.log 2>&1 || exit $?
timeout -k 10 300 $T -x -q tests/test_gpu_model.py -k "lstma or t120" > gpurun_out/c_modeltests.log 2>&1 || exit $?
for r in 1 2; do
  XCP_LSTM_PERSIST=0 timeout -k 10 200 python -u bench.py --model lstma --steps 20 --warmup 5 > gpurun_out/c_step_$r.log 2> gpurun_out/c_step_$r.err || exit $?
  timeout -k 10 200 python -u bench.py --model lstma --steps 20 --warmup 5 > gpurun_out/c_persist_$r.log 2> gpurun_out/c_persist_$r.err || exit $?
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/c_prof -o c -- python -u bench.py --model lstma --steps 10 --warmup 3 > gpurun_out/c_prof.log 2>&1 || exit $?
