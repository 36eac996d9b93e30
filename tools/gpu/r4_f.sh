# Round 4 (f): depthwise backward without the compiler's per-step vmcnt(0) drains: kernel tests,
# kernel A/B against the previous commit (tools/dw_ab.py), in-step A/B (XCP_LIB_PATH)
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest -p no:cacheprovider --timeout 300 --timeout-method thread -rf tests/test_gpu_kernels.py -q -k "dw_" > gpurun_out/f_tests.log 2>&1 || exit $?
timeout -k 10 300 python -u tools/dw_ab.py run > gpurun_out/f_dwab.log 2>&1 || exit $?
Q="--cpu-baseline off --mode unfrozen --small-batch 0 --measured-peaks off --diag off --no-kernel-timing"
for v in new old new old; do
  if [ $v = old ]; then E="XCP_LIB_PATH=tools/exp/dwold/libxcp.so"; else E=""; fi
  env $E timeout -k 10 200 python bench.py $Q > gpurun_out/f_step_$v.json 2>> gpurun_out/f_step.err || exit $?
  echo "$v $(cat gpurun_out/f_step_$v.json)" >> gpurun_out/f_step.log
done
