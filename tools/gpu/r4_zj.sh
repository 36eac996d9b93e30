# Round 4 (zj): conv1 forward on contiguous output-row ranges reusing the shared input row (input read once
# instead of 1.5 times): conv1 kernel tests, model tests, kernel times, in-step A/B against the strided-row
# kernel (XCP_LIB_PATH=tools/exp/c1old/libxcp.so), 3 rounds
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
( while true; do date >> gpurun_out/zj_heartbeat.txt; sleep 50; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
timeout -k 10 300 python -u -m pytest -p no:cacheprovider --timeout 150 --timeout-method thread -rf tests/test_gpu_kernels.py -q \
  -k "conv1" > gpurun_out/zj_tests.log 2>&1 || exit $?
timeout -k 10 600 python -u -m pytest -p no:cacheprovider --timeout 500 --timeout-method thread -rf -s tests/test_gpu_model.py -q > gpurun_out/zj_model.log 2>&1 || exit $?
for v in new old new old; do
  if [ $v = old ]; then E="XCP_LIB_PATH=$PWD/tools/exp/c1old/libxcp.so"; else E="XCP_NONE=1"; fi
  echo "== $v" >> gpurun_out/zj_kb.log
  env $E timeout -k 10 200 python -u tools/kbench.py conv1 >> gpurun_out/zj_kb.log 2>&1 || exit $?
done
Q="--cpu-baseline off --mode unfrozen --small-batch 0 --measured-peaks off --diag off --no-kernel-timing"
for r in 1 2 3; do
  for v in new old; do
    if [ $v = old ]; then E="XCP_LIB_PATH=$PWD/tools/exp/c1old/libxcp.so"; else E="XCP_NONE=1"; fi
    env $E timeout -k 10 240 python bench.py $Q > gpurun_out/zj_${v}_${r}.json 2>> gpurun_out/zj.err || exit $?
    echo "$v $(cat gpurun_out/zj_${v}_${r}.json)" >> gpurun_out/zj_step.log
  done
done
