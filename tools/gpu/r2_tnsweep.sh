# GPU: bench sweep of the weight-gradient GEMM's workgroup target (tools/exp/tn<v>) around the
# current library, one box.
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
B="python -u bench.py --steps 20 --warmup 5 --cpu-baseline off --measured-peaks off"
LIB=multimodal-deepfake-detection_amd/xcp/libxcp.so
cp $LIB /tmp/libxcp_cur.so
timeout -k 10 170 $B > gpurun_out/ts_cur1.json 2> gpurun_out/ts_cur1.err || exit $?
for v in "$@"; do
  cp tools/exp/tn$v/libxcp.so $LIB
  timeout -k 10 170 $B > gpurun_out/ts_$v.json 2> gpurun_out/ts_$v.err || { cp /tmp/libxcp_cur.so $LIB; exit 1; }
done
cp /tmp/libxcp_cur.so $LIB
timeout -k 10 170 $B > gpurun_out/ts_cur2.json 2> gpurun_out/ts_cur2.err
