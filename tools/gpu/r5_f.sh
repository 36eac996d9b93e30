# Round 5 (f3): folded vs partial-row BN finalizes at B = 64 with the partial-row path's fp32 pre-reduce of
# more than 2048 partial rows on (default) and off (XCP_FIN_MAX_ROWS=1000000)
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
XCP_FIN_MAX_ROWS=1000000 timeout -k 10 300 python -u tools/fold_ab.py 64 299 > gpurun_out/f_ab3.log 2>&1 || exit $?
