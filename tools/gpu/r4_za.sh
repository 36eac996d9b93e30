# Round 4 (za): the persistent NT kernel with pipelined fragment reads (XCP_NT_PIPE=1): bitwise tests, kernel times
# (tools/kbench.py ntprobe), in-step A/B (3 interleaved rounds)
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest -p no:cacheprovider --timeout 150 --timeout-method thread -rf tests/test_gpu_kernels.py -q \
  -k "pipelined_reads or persistent_bitwise or gemm_nt256 or entry_flow" > gpurun_out/za_tests.log 2>&1 || exit $?
XCP_NT_PIPE=1 timeout -k 10 300 python -u -m pytest -p no:cacheprovider --timeout 150 --timeout-method thread -rf tests/test_gpu_kernels.py -q \
  -k "persistent_bitwise or gemm_nt256 or entry_flow or gemm_nt_stats" > gpurun_out/za_tests_ph2.log 2>&1 || exit $?
for v in 0 1 0 1; do
  echo "== PIPE=$v" >> gpurun_out/za_kb.log
  XCP_NT_PIPE=$v timeout -k 10 120 python -u tools/kbench.py ntprobe >> gpurun_out/za_kb.log 2>&1 || exit $?
done
Q="--cpu-baseline off --mode unfrozen --small-batch 0 --measured-peaks off --diag off --no-kernel-timing"
for r in 1 2 3; do
  for v in 0 1; do
    XCP_NT_PIPE=$v timeout -k 10 240 python bench.py $Q > gpurun_out/za_${v}_${r}.json 2>> gpurun_out/z.err || exit $?
    echo "$v $(cat gpurun_out/za_${v}_${r}.json)" >> gpurun_out/za_step.log
  done
done
