# Round 3: in-step re-sweep of the weight-gradient GEMM's workgroup target after the depthwise changes
# (XCP_TN_TARGET_WGS, the side stream's CU share), 3 interleaved rounds; default 128
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
B="python bench.py --cpu-baseline off --mode unfrozen --small-batch 0 --measured-peaks off --steps 10 --warmup 3 --diag off"
for r in 1 2 3; do
  for v in 128 96 160 192; do
    XCP_TN_TARGET_WGS=$v timeout -k 10 240 $B > gpurun_out/tw_${v}_${r}.json 2> gpurun_out/tw_${v}_${r}.err || exit $?
    python - "$v" "$r" <<'PY'
import json, sys
d = json.loads(open(f"gpurun_out/tw_{sys.argv[1]}_{sys.argv[2]}.json").read().strip().splitlines()[-1])
print(f"XCP_TN_TARGET_WGS={int(sys.argv[1]):3d} round {sys.argv[2]}: {d['value']:.1f} clips/s  {d['ms_per_step']:.2f} ms", flush=True)
PY
  done
done
