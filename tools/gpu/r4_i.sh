# Round 4 (i): bf16 contract with engine realizations (median of 3) against the RMS of 24 autocast
# realizations: the model tests (prints every RHO); stem conv1 kernel times; in-step A/B of the conv1 fusions
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 200 python -u -m pytest -p no:cacheprovider --timeout 150 --timeout-method thread -rf tests/test_gpu_kernels.py -q \
  -k "conv1" > gpurun_out/i_tests.log 2>&1 || exit $?
timeout -k 10 900 python -u -m pytest -p no:cacheprovider --timeout 400 --timeout-method thread -rf -s tests/test_gpu_model.py -q > gpurun_out/i_model.log 2>&1
rc=$?; echo "model tests rc=$rc" >> gpurun_out/i_model.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 200 python -u tools/kbench.py conv1 conv2 > gpurun_out/i_kb.log 2>&1 || exit $?
Q="--cpu-baseline off --mode unfrozen --small-batch 0 --measured-peaks off --diag off --no-kernel-timing"
for r in 1 2; do
  for v in 11 00; do
    XCP_CONV1_BN_FUSED=${v:0:1} XCP_CONV1_STATS_FUSED=${v:1:1} timeout -k 10 200 python bench.py $Q > gpurun_out/i_step_${v}_${r}.json 2>> gpurun_out/i_step.err || exit $?
    echo "XCP_CONV1_BN_FUSED/STATS_FUSED=$v $(cat gpurun_out/i_step_${v}_${r}.json)" >> gpurun_out/i_step.log
  done
done
