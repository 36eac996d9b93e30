# Round 5 (c): pipelined depthwise forward: bitwise test vs the one-tile kernel, dw tests, the model
# tests that run it, kernel timing at the dw shapes (tools/kbench.py dwshapes), in-step A/B
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
T="python -u -m pytest -p no:cacheprovider --timeout 150 --timeout-method thread -rf"
timeout -k 10 300 $T -q tests/test_gpu_kernels.py -k "dw_fwd" > gpurun_out/c_tests.log 2>&1 || exit $?
timeout -k 10 600 $T -q tests/test_gpu_model.py tests/test_gpu_modules.py > gpurun_out/c_model.log 2>&1 || exit $?
for v in 1 0; do XCP_DW_FWD_PIPE=$v timeout -k 10 200 python tools/kbench.py dwshapes > gpurun_out/c_kb_$v.log 2>&1 || exit $?; done
Q="--cpu-baseline off --mode unfrozen --small-batch 0 --measured-peaks off --diag off --no-kernel-timing"
for r in 1 2; do
  for v in 1 0; do
    XCP_DW_FWD_PIPE=$v timeout -k 10 240 python bench.py $Q > gpurun_out/c_${v}_${r}.json 2>> gpurun_out/c.err || exit $?
    echo "$v $(cat gpurun_out/c_${v}_${r}.json)" >> gpurun_out/c_step.log
  done
done
