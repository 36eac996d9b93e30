# Round 3: depthwise forward with 8-B lanes (XCP_DW_FWD_W2=4 / 5: segment length): parity tests under
# each switch, step-shape kernel times with output fingerprints (bitwise comparison across processes),
# interleaved rounds
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
for v in 4 5; do
  XCP_DW_FWD_W2=$v timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_modules.py -m gpu -q --timeout 120 --timeout-method thread -p no:cacheprovider \
    -k "dw or separable or block" > gpurun_out/w2_t$v.log 2>&1
  rc=$?; echo "pytest rc=$rc" >> gpurun_out/w2_t$v.log
  if [ $rc -ne 0 ]; then exit $rc; fi
done
for r in 1 2; do
  for v in 0 4 5; do
    echo "== XCP_DW_FWD_W2=$v round $r"
    XCP_DW_FWD_W2=$v timeout -k 10 200 python -u tools/kbench.py dwshapes || exit $?
  done
done
