# Round 3: entry-flow forward pointwise GEMMs (K = 64-256) on the 128x128 kernel vs the 256x256 kernels
# (kbench entrygemm: tile 1 / 2 / 3 / auto), then in-step A/B of XCP_NT_BIG_MINK (smallest K for the
# automatic 256x256 choice: 384 default vs 64), interleaved
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u tools/kbench.py entrygemm > gpurun_out/eg_kb.log 2>&1 || exit $?
cat gpurun_out/eg_kb.log
XCP_NT_BIG_MINK=64 timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_model.py -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  -k "gemm_nt or bench_size" > gpurun_out/eg_t.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/eg_t.log
if [ $rc -ne 0 ]; then exit $rc; fi
B="python bench.py --cpu-baseline off --mode unfrozen --small-batch 0 --measured-peaks off --steps 10 --warmup 3 --diag off"
for r in 1 2 3; do
  for v in "384 128" "64 128" "384 192"; do
    set -- $v
    XCP_NT_BIG_MINK=$1 XCP_TN_TARGET_WGS=$2 timeout -k 10 240 $B > gpurun_out/eg_$1_$2_${r}.json 2> gpurun_out/eg_$1_$2_${r}.err || exit $?
    python - "$1" "$2" "$r" <<'PY'
import json, sys
k, t, r = sys.argv[1:4]
d = json.loads(open(f"gpurun_out/eg_{k}_{t}_{r}.json").read().strip().splitlines()[-1])
print(f"XCP_NT_BIG_MINK={int(k):3d} XCP_TN_TARGET_WGS={t} round {r}: {d['value']:.1f} clips/s  {d['ms_per_step']:.2f} ms", flush=True)
PY
  done
done
