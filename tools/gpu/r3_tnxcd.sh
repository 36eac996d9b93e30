# Round 3: weight-gradient GEMM split count a multiple of 8 (whole splits per XCD): TN parity tests
# and the bench-size step, then an in-step A/B (XCP_TN_XCD_SPLITS=0: the plain count), interleaved
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_model.py -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  -k "gemm_tn or bench_size or reduce_batch" > gpurun_out/tnx_t.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/tnx_t.log
if [ $rc -ne 0 ]; then exit $rc; fi
B="python bench.py --cpu-baseline off --mode unfrozen --small-batch 0 --measured-peaks off --steps 10 --warmup 3 --diag off"
for r in 1 2 3; do
  for v in 1 0; do
    XCP_TN_XCD_SPLITS=$v timeout -k 10 240 $B > gpurun_out/tnx_${v}_${r}.json 2> gpurun_out/tnx_${v}_${r}.err || exit $?
    python - "$v" "$r" <<'PY'
import json, sys
d = json.loads(open(f"gpurun_out/tnx_{sys.argv[1]}_{sys.argv[2]}.json").read().strip().splitlines()[-1])
print(f"XCP_TN_XCD_SPLITS={sys.argv[1]} round {sys.argv[2]}: {d['value']:.1f} clips/s  {d['ms_per_step']:.2f} ms", flush=True)
PY
  done
done
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmct_fetch -o p -- python bench.py --cpu-baseline off --mode unfrozen --steps 3 --warmup 1 --small-batch 0 --measured-peaks off --diag off --no-kernel-timing > gpurun_out/tnx_pmc.log 2>&1
