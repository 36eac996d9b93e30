# GPU: C5 (AU+face) line repeated: current / XCP_STEM_FUSED=0 / current / TN target 256 / current.
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
B="python -u bench.py --model auface --cpu-baseline off --steps 6 --warmup 2"
timeout -k 10 200 $B > gpurun_out/c5b_cur1.json 2> gpurun_out/c5b_cur1.err || exit $?
XCP_STEM_FUSED=0 timeout -k 10 200 $B > gpurun_out/c5b_nostem.json 2> gpurun_out/c5b_nostem.err || exit $?
timeout -k 10 200 $B > gpurun_out/c5b_cur2.json 2> gpurun_out/c5b_cur2.err || exit $?
LIB=multimodal-deepfake-detection_amd/xcp/libxcp.so
cp $LIB /tmp/libxcp_cur.so
cp tools/exp/tn256/libxcp.so $LIB
timeout -k 10 200 $B > gpurun_out/c5b_tn256.json 2> gpurun_out/c5b_tn256.err
rc=$?
cp /tmp/libxcp_cur.so $LIB
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 $B > gpurun_out/c5b_cur3.json 2> gpurun_out/c5b_cur3.err
