# Round 5 (g): the model / module / train-step / DDP suites with the folded finalizes, in-step A/B fold on / off,
# then the depthwise-forward ring-shape sweep (XCP_DW_FWD_PIPE)
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
T="python -u -m pytest -p no:cacheprovider --timeout 200 --timeout-method thread -rf"
timeout -k 10 900 $T -q tests/test_gpu_model.py tests/test_gpu_modules.py tests/test_gpu_train_step.py tests/test_gpu_ddp.py > gpurun_out/g_model.log 2>&1 || exit $?
Q="--cpu-baseline off --mode unfrozen --small-batch 0 --measured-peaks off --diag off --no-kernel-timing"
for r in 1 2; do
  for v in 1 0; do
    XCP_BN_FOLD=$v timeout -k 10 240 python bench.py $Q > gpurun_out/g_${v}_${r}.json 2>> gpurun_out/g.err || exit $?
    echo "$v $(cat gpurun_out/g_${v}_${r}.json)" >> gpurun_out/g_step.log
  done
done
for v in 0 1 2 3 4; do XCP_DW_FWD_PIPE=$v timeout -k 10 200 python tools/kbench.py dwshapes > gpurun_out/g_kb_$v.log 2>&1 || exit $?; done
