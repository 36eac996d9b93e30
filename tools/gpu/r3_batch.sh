# Round 3: reduce-batch test + full GPU suite, bench, NT phase stamps + A/B.
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r3_t4.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/r3_t4.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 --cpu-baseline off > gpurun_out/r3_b4.json 2> gpurun_out/r3_b4.err || exit $?
timeout -k 10 200 python -u tools/gemm_phase.py run > gpurun_out/r3_phase.log 2>&1 || exit $?
timeout -k 10 300 python -u tools/gemm_ab.py 5 > gpurun_out/r3_ab2.log 2>&1 || exit $?
