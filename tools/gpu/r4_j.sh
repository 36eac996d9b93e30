# Round 4 (j): stem conv1 row kernels on 16-B input loads / output stores, two LDS read batches per
# pixel in the weight gradient; stem conv2 (conv3x3) without the per-tile store drain: kernel tests, kernel times (kbench conv1 / conv2), in-step A/B
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 200 python -u -m pytest -p no:cacheprovider --timeout 150 --timeout-method thread -rf tests/test_gpu_kernels.py -q \
  -k "conv1 or conv3x3" > gpurun_out/j_tests.log 2>&1 || exit $?
timeout -k 10 200 python -u tools/kbench.py conv1 conv2 > gpurun_out/j_kb.log 2>&1 || exit $?
Q="--cpu-baseline off --mode unfrozen --small-batch 0 --measured-peaks off --diag off --no-kernel-timing"
for r in 1 2; do
  for v in 11 00; do
    XCP_CONV1_BN_FUSED=${v:0:1} XCP_CONV1_STATS_FUSED=${v:1:1} timeout -k 10 200 python bench.py $Q > gpurun_out/j_step_${v}_${r}.json 2>> gpurun_out/j_step.err || exit $?
    echo "XCP_CONV1_BN_FUSED/STATS_FUSED=$v $(cat gpurun_out/j_step_${v}_${r}.json)" >> gpurun_out/j_step.log
  done
done
