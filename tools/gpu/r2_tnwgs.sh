# GPU: bench A/B -- weight-gradient GEMM on half the CUs (tools/exp/tn128) vs current, then the
# side-stream switch (XCP_WGRAD_STREAM) on the current library.
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
B="python -u bench.py --steps 20 --warmup 5 --cpu-baseline off --measured-peaks off"
LIB=multimodal-deepfake-detection_amd/xcp/libxcp.so
cp $LIB /tmp/libxcp_cur.so
timeout -k 10 170 $B > gpurun_out/tw_cur1.json 2> gpurun_out/tw_cur1.err || exit $?
cp tools/exp/tn128/libxcp.so $LIB
timeout -k 10 170 $B > gpurun_out/tw_128.json 2> gpurun_out/tw_128.err
rc=$?
cp /tmp/libxcp_cur.so $LIB
[ $rc -eq 0 ] || exit $rc
timeout -k 10 170 $B > gpurun_out/tw_cur2.json 2> gpurun_out/tw_cur2.err || exit $?
XCP_WGRAD_STREAM=0 timeout -k 10 170 $B > gpurun_out/tw_ws0.json 2> gpurun_out/tw_ws0.err
