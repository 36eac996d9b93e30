# Round 3: A/Bs in one box: the weight-gradient GEMM's XCD-whole split count (XCP_TN_XCD_SPLITS=0: plain
# count), the depthwise backward streaming at one row of look-ahead (XCP_DW_BWD_OCC4=1: four waves per
# SIMD without a residual, three with one) and the depthwise forward with 8-B lanes (XCP_DW_FWD_W2=4/5);
# parity tests under the switches, kernel A/Bs (depthwise backward against the committed kernel; forward
# step shapes with output fingerprints), then in-step rounds
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
XCP_DW_BWD_OCC4=1 XCP_DW_FWD_W2=4 timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_modules.py tests/test_gpu_model.py -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  -k "gemm_tn or bench_size or reduce_batch or dw or block or separable" > gpurun_out/ab3_t.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/ab3_t.log
if [ $rc -ne 0 ]; then exit $rc; fi
XCP_DW_FWD_W2=5 timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -m gpu -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  -k "dw" > gpurun_out/ab3_t5.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/ab3_t5.log
if [ $rc -ne 0 ]; then exit $rc; fi
XCP_DW_BWD_OCC4=1 timeout -k 10 200 python -u tools/dw_ab.py run > gpurun_out/occ4_ab.log 2>&1 || exit $?
cat gpurun_out/occ4_ab.log
for r in 1 2; do
  for v in 0 4 5; do
    echo "== XCP_DW_FWD_W2=$v round $r"
    XCP_DW_FWD_W2=$v timeout -k 10 200 python -u tools/kbench.py dwshapes || exit $?
  done
done > gpurun_out/w2_kb.log 2>&1
B="python bench.py --cpu-baseline off --mode unfrozen --small-batch 0 --measured-peaks off --steps 10 --warmup 3 --diag off"
for r in 1 2 3; do
  for v in "1 0 0" "0 0 0" "1 1 0" "1 1 4"; do
    set -- $v
    XCP_TN_XCD_SPLITS=$1 XCP_DW_BWD_OCC4=$2 XCP_DW_FWD_W2=$3 timeout -k 10 240 $B > gpurun_out/ab3_$1$2$3_${r}.json 2> gpurun_out/ab3_$1$2$3_${r}.err || exit $?
    python - "$1" "$2" "$3" "$r" <<'PY'
import json, sys
x, o, w, r = sys.argv[1:5]
d = json.loads(open(f"gpurun_out/ab3_{x}{o}{w}_{r}.json").read().strip().splitlines()[-1])
print(f"XCD_SPLITS={x} DW_BWD_OCC4={o} DW_FWD_W2={w} round {r}: {d['value']:.1f} clips/s  {d['ms_per_step']:.2f} ms", flush=True)
PY
  done
done
