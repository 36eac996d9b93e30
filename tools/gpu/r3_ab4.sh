# Round 3: entry-flow GEMM tiles (kbench entrygemm), block-boundary BN sums from the depthwise backward
# (XCP_RESBN=1) parity tests, then in-step A/B of RESBN, XCP_NT_BIG_MINK=64 and XCP_TN_TARGET_WGS=192
# against the defaults, interleaved
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
XCP_RESBN=1 timeout -k 10 500 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_model.py tests/test_gpu_modules.py tests/test_gpu_train_step.py -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider -rf \
  > gpurun_out/ab4_t.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/ab4_t.log
tail -n 5 gpurun_out/ab4_t.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python -u tools/kbench.py entrygemm > gpurun_out/eg_kb.log 2>&1 || exit $?
B="python bench.py --cpu-baseline off --mode unfrozen --small-batch 0 --measured-peaks off --steps 10 --warmup 3 --diag off"
for r in 1 2 3; do
  for v in "0 384 128" "1 384 128" "0 64 128" "0 384 192"; do
    set -- $v
    XCP_RESBN=$1 XCP_NT_BIG_MINK=$2 XCP_TN_TARGET_WGS=$3 timeout -k 10 240 $B > gpurun_out/ab4_$1_$2_$3_${r}.json 2> gpurun_out/ab4_$1_$2_$3_${r}.err || exit $?
    python - "$1" "$2" "$3" "$r" <<'PY'
import json, sys
a, k, t, r = sys.argv[1:5]
d = json.loads(open(f"gpurun_out/ab4_{a}_{k}_{t}_{r}.json").read().strip().splitlines()[-1])
print(f"RESBN={a} NT_BIG_MINK={int(k):3d} TN_TARGET_WGS={t} round {r}: {d['value']:.1f} clips/s  {d['ms_per_step']:.2f} ms", flush=True)
PY
  done
done
