# GPU: XceptionLSTMA (C4) bench line and its rocprofv3 kernel trace + stats.
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 170 python -u bench.py --model lstma --cpu-baseline off > gpurun_out/lstma_b.json 2> gpurun_out/lstma_b.err || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_lstma -o kt -- python bench.py --model lstma --cpu-baseline off --steps 5 --warmup 2 --no-kernel-timing > gpurun_out/lstma_prof.log 2>&1
