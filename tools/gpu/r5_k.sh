# Round 5 (k): host-side timeline of the headline step (tools/host_timeline.py)
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u tools/host_timeline.py 4 > gpurun_out/k_host.log 2>&1 || exit $?
