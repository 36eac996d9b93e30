# Round 4 (n): the train step as one HIP graph: capture tests (optimiser, whole step vs eager, bitwise),
# bench graph on vs off (interleaved), kernel trace of the graph-replayed step
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest -p no:cacheprovider --timeout 200 --timeout-method thread -rf tests/test_gpu_train_step.py -v \
  -k "capturable or graph_captured or second_step" > gpurun_out/n_tests.log 2>&1 || exit $?
Q="--cpu-baseline off --mode unfrozen --small-batch 0 --measured-peaks off --diag off"
for r in 1 2; do
  for v in on off; do
    timeout -k 10 240 python bench.py $Q --graph $v > gpurun_out/n_step_${v}_${r}.json 2>> gpurun_out/n_step.err || exit $?
    echo "graph=$v $(cat gpurun_out/n_step_${v}_${r}.json)" >> gpurun_out/n_step.log
  done
done
B="python bench.py --cpu-baseline off --mode unfrozen --steps 5 --warmup 2 --small-batch 0 --measured-peaks off --diag off --no-kernel-timing"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_r4n -o kt -- $B > gpurun_out/n_prof.log 2>&1 || exit $?
python tools/stream_timeline.py "$(find gpurun_out/prof_r4n -name "*kernel_trace.csv" | head -1)" 40 > gpurun_out/n_timeline.txt 2>&1
