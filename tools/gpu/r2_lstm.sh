# GPU: LSTM parity tests, then the XceptionLSTMA bench line with the current library and with
# tools/exp/old (previous LSTM kernels), and the depthwise channel-slicing experiment.
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 200 python -u -m pytest -x -q --timeout 150 --timeout-method thread tests/test_gpu_kernels.py tests/test_gpu_model.py -k "lstm or audio" > gpurun_out/lstm_tests.log 2>&1 || exit $?
timeout -k 10 170 python -u bench.py --model lstma --cpu-baseline off > gpurun_out/lstm_new1.json 2> gpurun_out/lstm_new1.err || exit $?
cp multimodal-deepfake-detection_amd/xcp/libxcp.so /tmp/libxcp_cur.so
cp tools/exp/old/libxcp.so multimodal-deepfake-detection_amd/xcp/libxcp.so
timeout -k 10 170 python -u bench.py --model lstma --cpu-baseline off > gpurun_out/lstm_old.json 2> gpurun_out/lstm_old.err
rc=$?
cp /tmp/libxcp_cur.so multimodal-deepfake-detection_amd/xcp/libxcp.so
[ $rc -eq 0 ] || exit $rc
timeout -k 10 170 python -u bench.py --model lstma --cpu-baseline off > gpurun_out/lstm_new2.json 2> gpurun_out/lstm_new2.err || exit $?
timeout -k 10 200 python -u tools/kbench.py dwloc > gpurun_out/dwloc.log 2>&1
