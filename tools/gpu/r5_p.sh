# Round 5 (p): fused block1 forward probes (timing only): p1 no depthwise window reads / FMAs, p2 no MFMA,
# p3 no D / Y stores (issued out of range); base = shipped
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 200 python -u tools/sep_bench.py 10 > gpurun_out/p_base.log 2>&1 || exit $?
for v in p1 p2 p3; do
  XCP_LIB_PATH=probe/$v/libxcp.so timeout -k 10 200 python -u tools/sep_bench.py 10 > gpurun_out/p_$v.log 2>&1 || exit $?
done
