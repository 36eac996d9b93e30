# GPU: C4 (XceptionLSTMA) bench and a kernel trace of it (is the step launch-bound?).
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python bench.py --model lstma --cpu-baseline off > gpurun_out/r2_lstma.json 2> gpurun_out/r2_lstma.err || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_lstma -o kt -- python bench.py --model lstma --cpu-baseline off --steps 5 --warmup 2 > gpurun_out/r2_lstma_prof.log 2>&1
