# Round 4 (zh): the batched weight pack on 4-element groups (16-B loads, 8-B bf16 stores): pack tests, model
# tests, in-step A/B against the per-element pack (XCP_LIB_PATH=tools/exp/packold/libxcp.so), 3 rounds
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
( while true; do date >> gpurun_out/zh_heartbeat.txt; sleep 50; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
timeout -k 10 300 python -u -m pytest -p no:cacheprovider --timeout 150 --timeout-method thread -rf tests/test_gpu_kernels.py -q \
  -k "permute" > gpurun_out/zh_tests.log 2>&1 || exit $?
timeout -k 10 600 python -u -m pytest -p no:cacheprovider --timeout 500 --timeout-method thread -rf -s tests/test_gpu_model.py tests/test_gpu_train_step.py -q > gpurun_out/zh_model.log 2>&1 || exit $?
B="python bench.py --cpu-baseline off --mode unfrozen --steps 5 --warmup 2 --small-batch 0 --measured-peaks off --diag off --no-kernel-timing"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_zh -o kt -- $B > gpurun_out/zh_prof.log 2>&1 || exit $?
Q="--cpu-baseline off --mode unfrozen --small-batch 0 --measured-peaks off --diag off --no-kernel-timing"
for r in 1 2 3; do
  for v in new old; do
    if [ $v = old ]; then E="XCP_LIB_PATH=$PWD/tools/exp/packold/libxcp.so"; else E="XCP_NONE=1"; fi
    env $E timeout -k 10 240 python bench.py $Q > gpurun_out/zh_${v}_${r}.json 2>> gpurun_out/zh.err || exit $?
    echo "$v $(cat gpurun_out/zh_${v}_${r}.json)" >> gpurun_out/zh_step.log
  done
done
