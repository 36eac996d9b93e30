# GPU: GEMM ablation variants (tools/gemm_exp.py, prebuilt in tools/exp/).
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u tools/gemm_exp.py run > gpurun_out/r2_exp.log 2>&1
