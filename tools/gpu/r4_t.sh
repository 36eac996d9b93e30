# Round 4 (t): conv1 matrix-core kernels with split-bf16 (head + tail) products: kernel tests, kernel times,
# the model tests (bf16 contract, backbone64 feature cosine), in-step A/B against the fp32-FMA row kernels
# (XCP_LIB_PATH=tools/exp/stemvalu/libxcp.so)
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
( while true; do date >> gpurun_out/t_heartbeat.txt; sleep 50; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
timeout -k 10 200 python -u -m pytest -p no:cacheprovider --timeout 150 --timeout-method thread -rf tests/test_gpu_kernels.py -q \
  -k "conv1" > gpurun_out/t_tests.log 2>&1 || exit $?
timeout -k 10 200 python -u tools/kbench.py conv1 > gpurun_out/t_kb.log 2>&1 || exit $?
timeout -k 10 900 python -u -m pytest -p no:cacheprovider --timeout 500 --timeout-method thread -rf -s tests/test_gpu_model.py -q > gpurun_out/t_model.log 2>&1
rc=$?; echo "model tests rc=$rc" >> gpurun_out/t_model.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
Q="--cpu-baseline off --mode unfrozen --small-batch 0 --measured-peaks off --diag off --no-kernel-timing"
for r in 1 2; do
  for v in mfma valu; do
    if [ $v = valu ]; then E="XCP_LIB_PATH=$PWD/tools/exp/stemvalu/libxcp.so"; else E="XCP_NONE=1"; fi
    env $E timeout -k 10 240 python bench.py $Q > gpurun_out/t_step_${v}_${r}.json 2>> gpurun_out/t_step.err || exit $?
    echo "$v $(cat gpurun_out/t_step_${v}_${r}.json)" >> gpurun_out/t_step.log
  done
done
