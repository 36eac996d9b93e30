# Round 5 (l): fused depthwise + pointwise forward for block1 (csrc/sepfwd.hip): kernel tests, model tests,
# then in-step A/B (XCP_SEP_FUSED, 3 rounds alternating) and the per-op kbench of block1's forward
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
T="python -u -m pytest -p no:cacheprovider --timeout 200 --timeout-method thread -rf"
timeout -k 10 300 $T -x -q tests/test_gpu_kernels.py -k "sep_fwd" > gpurun_out/l_tests.log 2>&1 || exit $?
timeout -k 10 600 $T -q tests/test_gpu_model.py tests/test_gpu_train_step.py > gpurun_out/l_model.log 2>&1; echo "model rc=$?" >> gpurun_out/l_model.log
Q="--cpu-baseline off --mode unfrozen --small-batch 0 --measured-peaks off --diag off --no-kernel-timing"
for r in 1 2 3; do
  for v in 1 0; do
    XCP_SEP_FUSED=$v timeout -k 10 240 python bench.py $Q > gpurun_out/l_${v}_${r}.json 2>> gpurun_out/l.err || exit $?
    python -c "import json; d=json.load(open('gpurun_out/l_${v}_${r}.json')); print('$v', d['value'], d['ms_per_step'])" >> gpurun_out/l_step.log
  done
done
B="python bench.py --cpu-baseline off --mode unfrozen --steps 3 --warmup 2 --small-batch 0 --measured-peaks off --diag off --no-kernel-timing"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_r5l -o kt -- $B > gpurun_out/l_prof.log 2>&1 || exit $?
