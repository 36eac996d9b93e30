# GPU: one kbench run.  usage: bash tools/gpu/r2_kb.sh "<kbench names>" <log name>
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 170 python -u tools/kbench.py $1 > gpurun_out/$2.log 2>&1
