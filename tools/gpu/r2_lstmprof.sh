# GPU: rocprofv3 kernel trace of the XceptionLSTMA line, current build vs tools/exp/lstmold
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
LIB=multimodal-deepfake-detection_amd/xcp/libxcp.so
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/lsp_new -o kt -- python3 -u bench.py --model lstma \
  --steps 5 --warmup 2 --cpu-baseline off --measured-peaks off > gpurun_out/lsp_new.log 2>&1 || exit $?
cp $LIB /tmp/libxcp_cur.so
cp tools/exp/lstmold/libxcp.so $LIB
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/lsp_old -o kt -- python3 -u bench.py --model lstma \
  --steps 5 --warmup 2 --cpu-baseline off --measured-peaks off > gpurun_out/lsp_old.log 2>&1
rc=$?
cp /tmp/libxcp_cur.so $LIB
exit $rc
