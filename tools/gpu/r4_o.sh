# Round 4 (o): host vs device time per phase of the headline step (tools/cpu_overhead.py)
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 200 python -u tools/cpu_overhead.py > gpurun_out/o_cpu.log 2>&1 || exit $?
