# Round 3: in-step A/B, interleaved: current (batched slab reductions + BN1 coefficients before the
# side-stream conv2 weight gradient), XCP_REDUCE_BATCH=0, XCP_STEM_BN1_FIRST=0
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
B="python bench.py --cpu-baseline off --mode unfrozen --small-batch 0 --measured-peaks off --steps 10 --warmup 3"
for r in 1 2 3; do
  for v in cur nobatch bn1late; do
    case $v in
      cur) E="";;
      nobatch) E="XCP_REDUCE_BATCH=0";;
      bn1late) E="XCP_STEM_BN1_FIRST=0";;
    esac
    env $E timeout -k 10 240 $B > gpurun_out/sab_${v}_r${r}.json 2> gpurun_out/sab_${v}_r${r}.err || exit $?
    python - "$v" "$r" <<'PY'
import json, sys
d = json.loads(open(f"gpurun_out/sab_{sys.argv[1]}_r{sys.argv[2]}.json").read().strip().splitlines()[-1])
u = d["diag"]["unfrozen"]
print(f"{sys.argv[1]:8s} round {sys.argv[2]}: {d['value']:.1f} clips/s  {d['ms_per_step']:.2f} ms  fwd {u['fwd_ms']:.2f} bwd {u['bwd_ms']:.2f}", flush=True)
PY
  done
done
timeout -k 10 120 python -u tools/kbench.py chanred fin > gpurun_out/sab_kbench.log 2>&1
