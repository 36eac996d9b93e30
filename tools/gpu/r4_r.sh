# Round 4 (r): block-boundary BN sums from the depthwise backward (XCP_RESBN=1) vs the per-channel
# reduce, interleaved x3 (no kernel timer, no diag)
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
Q="--cpu-baseline off --mode unfrozen --small-batch 0 --measured-peaks off --diag off --no-kernel-timing"
for r in 1 2 3; do
  for v in 0 1; do
    XCP_RESBN=$v timeout -k 10 240 python bench.py $Q > gpurun_out/r_step_${v}_${r}.json 2>> gpurun_out/r_step.err || exit $?
    echo "XCP_RESBN=$v $(cat gpurun_out/r_step_${v}_${r}.json)" >> gpurun_out/r_step.log
  done
done
timeout -k 10 300 python -u -m pytest -p no:cacheprovider --timeout 200 --timeout-method thread -rf tests/test_gpu_kernels.py -q -k "resbn or dw_bwd" > gpurun_out/r_tests.log 2>&1 || exit $?
