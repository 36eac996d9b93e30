# GPU: tiny-frame depthwise forward A/B -- rows fetched one step ahead with no per-load branch
# (current build) vs the per-load-branch version (tools/exp/dwsold): kbench dwsmall and the
# XceptionLSTMA line, after the depthwise parity tests.
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
LIB=multimodal-deepfake-detection_amd/xcp/libxcp.so
B="python -u bench.py --model lstma --steps 30 --warmup 5 --cpu-baseline off --measured-peaks off"
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py -x -v --timeout 120 --timeout-method thread -m gpu \
  -k "dw_fwd_bwd" > gpurun_out/ds_tests.log 2>&1 || exit $?
timeout -k 10 120 python -u tools/kbench.py dwsmall > gpurun_out/ds_new1.txt 2>&1 || exit $?
timeout -k 10 170 $B > gpurun_out/ds_new1.json 2> gpurun_out/ds_new1.err || exit $?
cp $LIB /tmp/libxcp_cur.so
cp tools/exp/dwsold/libxcp.so $LIB
timeout -k 10 120 python -u tools/kbench.py dwsmall > gpurun_out/ds_old.txt 2>&1 && \
  timeout -k 10 170 $B > gpurun_out/ds_old.json 2> gpurun_out/ds_old.err
rc=$?
cp /tmp/libxcp_cur.so $LIB
[ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -u tools/kbench.py dwsmall > gpurun_out/ds_new2.txt 2>&1 || exit $?
timeout -k 10 170 $B > gpurun_out/ds_new2.json 2> gpurun_out/ds_new2.err
