# GPU: max-pool backward + BN reduce A/B -- software-pipelined quad loop (current build) vs one
# dependent round trip per quad (tools/exp/poolold): tail / pool tests, kbench poolbwd, bench.
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
LIB=multimodal-deepfake-detection_amd/xcp/libxcp.so
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -v --timeout 120 --timeout-method thread -m gpu \
  -k "tail or pool" > gpurun_out/pb_tests.log 2>&1 || exit $?
timeout -k 10 120 python -u tools/kbench.py poolbwd > gpurun_out/pb_new1.txt 2>&1 || exit $?
cp $LIB /tmp/libxcp_cur.so
cp tools/exp/poolold/libxcp.so $LIB
timeout -k 10 120 python -u tools/kbench.py poolbwd > gpurun_out/pb_old.txt 2>&1
rc=$?
cp /tmp/libxcp_cur.so $LIB
[ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -u tools/kbench.py poolbwd > gpurun_out/pb_new2.txt 2>&1 || exit $?
timeout -k 10 170 python -u bench.py --steps 20 --warmup 5 --cpu-baseline off --measured-peaks off \
  > gpurun_out/pb_bench.json 2> gpurun_out/pb_bench.err
