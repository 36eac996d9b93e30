# Round 4 (zc): the 128x128 NT kernel with a 3-stage LDS ring (XCP_NT_STAGES=3; the persistent kernel's
# sparse last round and every 128x128 NT launch): bitwise tests, op times, in-step A/B (3 interleaved rounds)
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest -p no:cacheprovider --timeout 150 --timeout-method thread -rf tests/test_gpu_kernels.py -q \
  -k "three_stage or gemm_nt" > gpurun_out/zc_tests.log 2>&1 || exit $?
XCP_NT_STAGES=3 timeout -k 10 300 python -u -m pytest -p no:cacheprovider --timeout 150 --timeout-method thread -rf tests/test_gpu_kernels.py -q \
  -k "gemm_nt" > gpurun_out/zc_tests3.log 2>&1 || exit $?
for v in 2 3 2 3; do
  echo "== STAGES=$v" >> gpurun_out/zc_kb.log
  XCP_NT_STAGES=$v timeout -k 10 120 python -u tools/kbench.py ntprobe entrygemm >> gpurun_out/zc_kb.log 2>&1 || exit $?
done
Q="--cpu-baseline off --mode unfrozen --small-batch 0 --measured-peaks off --diag off --no-kernel-timing"
for r in 1 2 3; do
  for v in 2 3; do
    XCP_NT_STAGES=$v timeout -k 10 240 python bench.py $Q > gpurun_out/zc_${v}_${r}.json 2>> gpurun_out/zc.err || exit $?
    echo "$v $(cat gpurun_out/zc_${v}_${r}.json)" >> gpurun_out/zc_step.log
  done
done
