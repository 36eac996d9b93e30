# Round 3: in-step A/B of the big pointwise GEMM kernel choice (XCP_NT_TILE: 0 persistent 8-wave,
# 4 one-shot 8-wave), interleaved, unfrozen headline step only
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
B="python bench.py --cpu-baseline off --mode unfrozen --small-batch 0 --measured-peaks off --steps 10 --warmup 3"
for r in 1 2 3; do
  for t in 0 4; do
    XCP_NT_TILE=$t timeout -k 10 240 $B > gpurun_out/ntab_t${t}_r${r}.json 2> gpurun_out/ntab_t${t}_r${r}.err || exit $?
    python - "$t" "$r" <<'PY'
import json, sys
d = json.loads(open(f"gpurun_out/ntab_t{sys.argv[1]}_r{sys.argv[2]}.json").read().strip().splitlines()[-1])
print(f"tile {sys.argv[1]} round {sys.argv[2]}: {d['value']:.1f} clips/s  {d['ms_per_step']:.2f} ms  roofline {d['roofline']['avg_launch_ms']*1e3:.1f} us "
      f"fwd {d['diag']['unfrozen']['fwd_ms']:.2f} bwd {d['diag']['unfrozen']['bwd_ms']:.2f}", flush=True)
PY
  done
done
