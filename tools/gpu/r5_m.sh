# Round 5 (m): fused block1 forward vs two kernels on the 64^2 backbone (tools/sep_diag.py)
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u tools/sep_diag.py > gpurun_out/m_diag.log 2>&1 || exit $?
