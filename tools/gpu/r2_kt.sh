# GPU: rocprofv3 kernel trace + stats of the unfrozen bench (no PMC), weight gradients on the
# side stream (kt) and in order on the main stream (kt_ws0, isolated kernel durations).
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
B="python bench.py --cpu-baseline off --mode unfrozen --steps 7 --warmup 2"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_kt -o kt -- $B > gpurun_out/r2_kt.log 2>&1 || exit $?
XCP_WGRAD_STREAM=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_kt_ws0 -o kt -- $B > gpurun_out/r2_kt_ws0.log 2>&1 || exit $?
echo ok
