# Round 4 (zf): BN finalize kernels held to 72 VGPRs (fit beside the stem conv2 weight gradient): BN kernel
# tests, a kernel trace of the step (is BN1's backward finalize still blocked?), in-step A/B against the
# 108-VGPR kernels (XCP_LIB_PATH=tools/exp/finold/libxcp.so), 3 interleaved rounds
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest -p no:cacheprovider --timeout 150 --timeout-method thread -rf tests/test_gpu_kernels.py -q \
  -k "bn or finalize or stats" > gpurun_out/zf_tests.log 2>&1 || exit $?
B="python bench.py --cpu-baseline off --mode unfrozen --steps 5 --warmup 2 --small-batch 0 --measured-peaks off --diag off --no-kernel-timing"
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof_zf -o kt -- $B > gpurun_out/zf_prof.log 2>&1 || exit $?
Q="--cpu-baseline off --mode unfrozen --small-batch 0 --measured-peaks off --diag off --no-kernel-timing"
for r in 1 2 3; do
  for v in new old; do
    if [ $v = old ]; then E="XCP_LIB_PATH=$PWD/tools/exp/finold/libxcp.so"; else E="XCP_NONE=1"; fi
    env $E timeout -k 10 240 python bench.py $Q > gpurun_out/zf_${v}_${r}.json 2>> gpurun_out/zf.err || exit $?
    echo "$v $(cat gpurun_out/zf_${v}_${r}.json)" >> gpurun_out/zf_step.log
  done
done
