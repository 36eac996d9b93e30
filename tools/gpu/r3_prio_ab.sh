# Round 3: stream-priority A/B, interleaved: default; XCP_SIDE_PRIO=low (weight-gradient stream at the
# least priority); XCP_BENCH_STREAM=high (the step on a high-priority stream, side stream default)
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
B="python bench.py --cpu-baseline off --mode unfrozen --small-batch 0 --measured-peaks off --steps 10 --warmup 3"
for r in 1 2 3; do
  for v in def sidelow mainhigh; do
    case $v in
      def) E="";;
      sidelow) E="XCP_SIDE_PRIO=low";;
      mainhigh) E="XCP_BENCH_STREAM=high";;
    esac
    env $E timeout -k 10 240 $B > gpurun_out/pab_${v}_r${r}.json 2> gpurun_out/pab_${v}_r${r}.err || exit $?
    python - "$v" "$r" <<'PY'
import json, sys
d = json.loads(open(f"gpurun_out/pab_{sys.argv[1]}_r{sys.argv[2]}.json").read().strip().splitlines()[-1])
u = d["diag"]["unfrozen"]
print(f"{sys.argv[1]:8s} round {sys.argv[2]}: {d['value']:.1f} clips/s  {d['ms_per_step']:.2f} ms  fwd {u['fwd_ms']:.2f} bwd {u['bwd_ms']:.2f}  prio range {d['diag'].get('stream_priority_range')}", flush=True)
PY
  done
done
