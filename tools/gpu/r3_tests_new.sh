# Round 3: the new parity tests with their printed errors, the NT256 fixed-cost probe, then the whole GPU suite.
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest tests -m gpu -v -s --timeout 300 --timeout-method thread -p no:cacheprovider \
  -k "bench_size or frame_step or two_rank or dataparallel or resume" > gpurun_out/r3_new.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/r3_new.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -u tools/gemm_probe.py > gpurun_out/r3_probe.log 2>&1 || exit $?
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r3_t3.log 2>&1
echo "pytest rc=$?" >> gpurun_out/r3_t3.log
