# Round 5 (n): fused block1 forward -- kernel tests, per-launch bench (tools/sep_bench.py), SQ counters
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
T="python -u -m pytest -p no:cacheprovider --timeout 200 --timeout-method thread -rf"
timeout -k 10 300 $T -x -q tests/test_gpu_kernels.py -k "sep_fwd" > gpurun_out/n_tests.log 2>&1 || exit $?
timeout -k 10 300 python -u tools/sep_bench.py 10 > gpurun_out/n_bench.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES --output-format csv -d gpurun_out/n_pmc1 -o p -- python tools/sep_bench.py 2 > gpurun_out/n_pmc1.log 2>&1 || exit $?
