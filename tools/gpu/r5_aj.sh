# Round 5 (aj): the weight-gradient GEMM's workgroup target (XCP_TN_TARGET_WGS) re-swept with the NT tile
# queue in the input-gradient GEMMs: 96 / 128 (default) / 192, 3 interleaved rounds
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for r in 1 2 3; do
  for t in 128 96 192; do
    XCP_TN_TARGET_WGS=$t timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 > gpurun_out/aj_t${t}_$r.log 2> gpurun_out/aj_t${t}_$r.err || exit $?
  done
done
