# Round 3: block-boundary BN partial sums from the next block's first depthwise backward
# (xcp_dw_bwd_resbn; XCP_RESBN=0: the per-channel reduce): kernel + model parity tests, then in-step A/B
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
XCP_RESBN=1 timeout -k 10 500 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_model.py tests/test_gpu_modules.py tests/test_gpu_train_step.py -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider -rf \
  > gpurun_out/rb_t.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/rb_t.log
tail -n 5 gpurun_out/rb_t.log
if [ $rc -ne 0 ]; then exit $rc; fi
B="python bench.py --cpu-baseline off --mode unfrozen --small-batch 0 --measured-peaks off --steps 10 --warmup 3 --diag off"
for r in 1 2 3; do
  for v in 1 0; do
    XCP_RESBN=$v timeout -k 10 240 $B > gpurun_out/rb_${v}_${r}.json 2> gpurun_out/rb_${v}_${r}.err || exit $?
    python - "$v" "$r" <<'PY'
import json, sys
d = json.loads(open(f"gpurun_out/rb_{sys.argv[1]}_{sys.argv[2]}.json").read().strip().splitlines()[-1])
print(f"XCP_RESBN={sys.argv[1]} round {sys.argv[2]}: {d['value']:.1f} clips/s  {d['ms_per_step']:.2f} ms", flush=True)
PY
  done
done
