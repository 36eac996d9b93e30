# Round 4 (zg): the stem BNs' backward finalize on 4-wave workgroups (fits beside the side stream's stem conv2
# weight gradient): BN kernel tests, the model tests, a kernel trace of the step, in-step A/B against
# XCP_FIN4_SMALL=0 (16-wave workgroups), 3 interleaved rounds
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
( while true; do date >> gpurun_out/zg_heartbeat.txt; sleep 50; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
timeout -k 10 300 python -u -m pytest -p no:cacheprovider --timeout 150 --timeout-method thread -rf tests/test_gpu_kernels.py -q \
  -k "bn or finalize or stats or stem or conv" > gpurun_out/zg_tests.log 2>&1 || exit $?
timeout -k 10 600 python -u -m pytest -p no:cacheprovider --timeout 500 --timeout-method thread -rf -s tests/test_gpu_model.py -q > gpurun_out/zg_model.log 2>&1 || exit $?
B="python bench.py --cpu-baseline off --mode unfrozen --steps 5 --warmup 2 --small-batch 0 --measured-peaks off --diag off --no-kernel-timing"
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof_zg -o kt -- $B > gpurun_out/zg_prof.log 2>&1 || exit $?
Q="--cpu-baseline off --mode unfrozen --small-batch 0 --measured-peaks off --diag off --no-kernel-timing"
for r in 1 2 3; do
  for v in 1 0; do
    XCP_FIN4_SMALL=$v timeout -k 10 240 python bench.py $Q > gpurun_out/zg_${v}_${r}.json 2>> gpurun_out/zg.err || exit $?
    echo "$v $(cat gpurun_out/zg_${v}_${r}.json)" >> gpurun_out/zg_step.log
  done
done
