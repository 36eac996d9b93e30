# Round 4 (h): stem conv1 as row kernels: forward with BN1's statistics fused (xcp_conv1_fwd_stats), weight
# gradient with BN1's backward apply fused (xcp_conv1_wgrad_bn): kernel tests, model tests, kernel times
# (kbench conv1 / conv2), in-step A/B (XCP_CONV1_BN_FUSED / XCP_CONV1_STATS_FUSED)
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 200 python -u -m pytest -p no:cacheprovider --timeout 150 --timeout-method thread -rf tests/test_gpu_kernels.py -q \
  -k "conv1" > gpurun_out/h_tests.log 2>&1 || exit $?
timeout -k 10 200 python -u tools/kbench.py conv1 conv2 > gpurun_out/h_kb.log 2>&1 || exit $?
timeout -k 10 600 python -u -m pytest -p no:cacheprovider --timeout 300 --timeout-method thread -rf tests/test_gpu_model.py -q -x > gpurun_out/h_model.log 2>&1 || exit $?
Q="--cpu-baseline off --mode unfrozen --small-batch 0 --measured-peaks off --diag off --no-kernel-timing"
for r in 1 2; do
  for v in 11 00; do
    XCP_CONV1_BN_FUSED=${v:0:1} XCP_CONV1_STATS_FUSED=${v:1:1} timeout -k 10 200 python bench.py $Q > gpurun_out/h_step_${v}_${r}.json 2>> gpurun_out/h_step.err || exit $?
    echo "XCP_CONV1_BN_FUSED/STATS_FUSED=$v $(cat gpurun_out/h_step_${v}_${r}.json)" >> gpurun_out/h_step.log
  done
done
