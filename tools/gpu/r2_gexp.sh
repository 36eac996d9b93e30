# GPU: GEMM ablation variants (tools/gemm_exp.py; GEMM_EXP_VARIANTS selects).
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
GEMM_EXP_VARIANTS="$1" timeout -k 10 170 python -u tools/gemm_exp.py run > gpurun_out/gexp.log 2>&1
