# Round 3: two A/Bs in one box: the weight-gradient GEMM's XCD-whole split count (XCP_TN_XCD_SPLITS=0:
# plain count) and the depthwise backward at four waves per SIMD (XCP_DW_BWD_OCC4=1); parity tests
# under both switches, the depthwise kernel A/B against the committed kernel, then in-step rounds
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
XCP_DW_BWD_OCC4=1 timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_modules.py tests/test_gpu_model.py -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  -k "gemm_tn or bench_size or reduce_batch or dw or block or separable" > gpurun_out/ab2_t.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/ab2_t.log
if [ $rc -ne 0 ]; then exit $rc; fi
XCP_DW_BWD_OCC4=1 timeout -k 10 200 python -u tools/dw_ab.py run > gpurun_out/occ4_ab.log 2>&1 || exit $?
cat gpurun_out/occ4_ab.log
B="python bench.py --cpu-baseline off --mode unfrozen --small-batch 0 --measured-peaks off --steps 10 --warmup 3 --diag off"
for r in 1 2 3; do
  for v in "1 0" "0 0" "1 1"; do
    set -- $v
    XCP_TN_XCD_SPLITS=$1 XCP_DW_BWD_OCC4=$2 timeout -k 10 240 $B > gpurun_out/ab2_$1$2_${r}.json 2> gpurun_out/ab2_$1$2_${r}.err || exit $?
    python - "$1" "$2" "$r" <<'PY'
import json, sys
x, o, r = sys.argv[1:4]
d = json.loads(open(f"gpurun_out/ab2_{x}{o}_{r}.json").read().strip().splitlines()[-1])
print(f"XCP_TN_XCD_SPLITS={x} XCP_DW_BWD_OCC4={o} round {r}: {d['value']:.1f} clips/s  {d['ms_per_step']:.2f} ms", flush=True)
PY
  done
done
