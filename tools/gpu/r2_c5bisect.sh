# GPU: C5 (AU+face) line under each A/B switch and the weight-gradient target 256 variant.
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
B="python -u bench.py --model auface --cpu-baseline off --steps 6 --warmup 2"
timeout -k 10 200 $B > gpurun_out/c5_cur.json 2> gpurun_out/c5_cur.err || exit $?
XCP_STEM_FUSED=0 timeout -k 10 200 $B > gpurun_out/c5_nostem.json 2> gpurun_out/c5_nostem.err || exit $?
XCP_WGRAD_STREAM=0 timeout -k 10 200 $B > gpurun_out/c5_ws0.json 2> gpurun_out/c5_ws0.err || exit $?
LIB=multimodal-deepfake-detection_amd/xcp/libxcp.so
cp $LIB /tmp/libxcp_cur.so
cp tools/exp/tn256/libxcp.so $LIB
timeout -k 10 200 $B > gpurun_out/c5_tn256.json 2> gpurun_out/c5_tn256.err
rc=$?
cp /tmp/libxcp_cur.so $LIB
exit $rc
