# Round 3: depthwise backward (no residual, no skip input) with one row of look-ahead at four waves
# per SIMD (XCP_DW_BWD_OCC4=1): kernel parity tests under the switch, kernel A/B against the committed
# kernel, in-step A/B, interleaved
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
XCP_DW_BWD_OCC4=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_modules.py -m gpu -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  -k "dw or block or separable" > gpurun_out/occ4_t.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/occ4_t.log
if [ $rc -ne 0 ]; then exit $rc; fi
XCP_DW_BWD_OCC4=1 timeout -k 10 200 python -u tools/dw_ab.py run > gpurun_out/occ4_ab.log 2>&1 || exit $?
B="python bench.py --cpu-baseline off --mode unfrozen --small-batch 0 --measured-peaks off --steps 10 --warmup 3 --diag off"
for r in 1 2 3; do
  for v in 0 1; do
    XCP_DW_BWD_OCC4=$v timeout -k 10 240 $B > gpurun_out/occ4_${v}_${r}.json 2> gpurun_out/occ4_${v}_${r}.err || exit $?
    python - "$v" "$r" <<'PY'
import json, sys
d = json.loads(open(f"gpurun_out/occ4_{sys.argv[1]}_{sys.argv[2]}.json").read().strip().splitlines()[-1])
print(f"XCP_DW_BWD_OCC4={sys.argv[1]} round {sys.argv[2]}: {d['value']:.1f} clips/s  {d['ms_per_step']:.2f} ms", flush=True)
PY
  done
done
