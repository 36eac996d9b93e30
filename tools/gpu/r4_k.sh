# Round 4 (k): stem kernels (conv1 row kernels on 16-B loads / stores, conv3x3 without the per-tile store
# drain): kernel tests, kernel times; conv1.weight's bf16 error per stem path (tools/conv1_err.py);
# the model tests under the reworked bf16 contract; in-step A/B of the conv1 fusions
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
( while true; do date >> gpurun_out/k_heartbeat.txt; sleep 50; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
timeout -k 10 200 python -u -m pytest -p no:cacheprovider --timeout 150 --timeout-method thread -rf tests/test_gpu_kernels.py -q \
  -k "conv1 or conv3x3" > gpurun_out/k_tests.log 2>&1 || exit $?
timeout -k 10 200 python -u tools/kbench.py conv1 conv2 > gpurun_out/k_kb.log 2>&1 || exit $?
timeout -k 10 100 python -u tools/conv1_err.py >> gpurun_out/k_conv1err.log 2>&1 || exit $?
XCP_CONV1_BN_FUSED=0 timeout -k 10 100 python -u tools/conv1_err.py >> gpurun_out/k_conv1err.log 2>&1 || exit $?
XCP_CONV1_STATS_FUSED=0 timeout -k 10 100 python -u tools/conv1_err.py >> gpurun_out/k_conv1err.log 2>&1 || exit $?
XCP_CONV1_BN_FUSED=0 XCP_CONV1_STATS_FUSED=0 timeout -k 10 100 python -u tools/conv1_err.py >> gpurun_out/k_conv1err.log 2>&1 || exit $?
XCP_LIB_PATH=$PWD/tools/exp/dwold/libxcp.so XCP_CONV1_BN_FUSED=0 XCP_CONV1_STATS_FUSED=0 timeout -k 10 100 python -u tools/conv1_err.py >> gpurun_out/k_conv1err.log 2>&1 || exit $?
timeout -k 10 1000 python -u -m pytest -p no:cacheprovider --timeout 500 --timeout-method thread -rf -s -v tests/test_gpu_model.py > gpurun_out/k_model.log 2>&1
rc=$?; echo "model tests rc=$rc" >> gpurun_out/k_model.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
Q="--cpu-baseline off --mode unfrozen --small-batch 0 --measured-peaks off --diag off --no-kernel-timing"
for r in 1 2; do
  for v in 11 00; do
    XCP_CONV1_BN_FUSED=${v:0:1} XCP_CONV1_STATS_FUSED=${v:1:1} timeout -k 10 200 python bench.py $Q > gpurun_out/k_step_${v}_${r}.json 2>> gpurun_out/k_step.err || exit $?
    echo "XCP_CONV1_BN_FUSED/STATS_FUSED=$v $(cat gpurun_out/k_step_${v}_${r}.json)" >> gpurun_out/k_step.log
  done
done
