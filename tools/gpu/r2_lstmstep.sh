# GPU: per-step LSTM kernels A/B -- unconditional (clamped / stand-in) loads in the h staging, the
# W_hh column staging and the cells (current build) vs one round trip per conditional load
# (tools/exp/lstmold): LSTM parity tests, then the XceptionLSTMA line per library.
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
LIB=multimodal-deepfake-detection_amd/xcp/libxcp.so
B="python -u bench.py --model lstma --steps 30 --warmup 5 --cpu-baseline off --measured-peaks off"
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_model.py -x -v --timeout 120 \
  --timeout-method thread -m gpu -k "lstm" > gpurun_out/ls_tests.log 2>&1 || exit $?
timeout -k 10 170 $B > gpurun_out/ls_new1.json 2> gpurun_out/ls_new1.err || exit $?
cp $LIB /tmp/libxcp_cur.so
cp tools/exp/lstmold/libxcp.so $LIB
timeout -k 10 170 $B > gpurun_out/ls_old.json 2> gpurun_out/ls_old.err
rc=$?
cp /tmp/libxcp_cur.so $LIB
[ $rc -eq 0 ] || exit $rc
timeout -k 10 170 $B > gpurun_out/ls_new2.json 2> gpurun_out/ls_new2.err
