# Round 4 (p): does the per-op HIP-event timer perturb the headline? bench with / without kernel timing,
# interleaved x3, and a kernel trace of the step without it
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
Q="--cpu-baseline off --mode unfrozen --small-batch 0 --measured-peaks off --diag off"
for r in 1 2 3; do
  for v in timer none; do
    if [ $v = none ]; then E="--no-kernel-timing"; else E=""; fi
    timeout -k 10 240 python bench.py $Q $E > gpurun_out/p_step_${v}_${r}.json 2>> gpurun_out/p_step.err || exit $?
    echo "$v $(cat gpurun_out/p_step_${v}_${r}.json)" >> gpurun_out/p_step.log
  done
done
B="python bench.py --cpu-baseline off --mode unfrozen --steps 5 --warmup 2 --small-batch 0 --measured-peaks off --diag off --no-kernel-timing"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_r4p -o kt -- $B > gpurun_out/p_prof.log 2>&1 || exit $?
python tools/stream_timeline.py "$(find gpurun_out/prof_r4p -name "*kernel_trace.csv" | head -1)" 40 > gpurun_out/p_timeline.txt 2>&1
