# GPU: rocprofv3 kernel trace + stats of the unfrozen bench (no PMC).
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
B="python bench.py --cpu-baseline off --mode unfrozen --steps 7 --warmup 2"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_kt -o kt -- $B > gpurun_out/r2_kt.log 2>&1 || exit $?
echo ok
