# Round 5 (h): PRE2 persistent NT GEMM -- the NT GEMM tests with PRE2 on, the interleaved kernel A/B,
# then in-step A/B (2 rounds each, alternating)
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
T="python -u -m pytest -p no:cacheprovider --timeout 200 --timeout-method thread -rf"
XCP_NT_PRE2=1 timeout -k 10 300 $T -q tests/test_gpu_kernels.py -k "gemm_nt" > gpurun_out/h_tests.log 2>&1 || exit $?
timeout -k 10 300 python -u tools/nt_pre2_ab.py 5 > gpurun_out/h_ab.log 2>&1 || exit $?
Q="--cpu-baseline off --mode unfrozen --small-batch 0 --measured-peaks off --diag off --no-kernel-timing"
for r in 1 2; do
  for v in 1 0; do
    XCP_NT_PRE2=$v timeout -k 10 240 python bench.py $Q > gpurun_out/h_${v}_${r}.json 2>> gpurun_out/h.err || exit $?
    echo "$v $(cat gpurun_out/h_${v}_${r}.json)" >> gpurun_out/h_step.log
  done
done
