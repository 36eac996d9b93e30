# Round 5 (ak): knobs first measured before the NT tile queue, re-measured with it: the smallest K given the
# 256x256 NT kernel (XCP_NT_BIG_MINK 384 default / 256 / 128) and whole weight-gradient splits per XCD
# (XCP_TN_XCD_ALIGN=1), 3 interleaved rounds
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for r in 1 2 3; do
  timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 > gpurun_out/ak_def_$r.log 2> gpurun_out/ak_def_$r.err || exit $?
  XCP_NT_BIG_MINK=256 timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 > gpurun_out/ak_k256_$r.log 2> gpurun_out/ak_k256_$r.err || exit $?
  XCP_NT_BIG_MINK=128 timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 > gpurun_out/ak_k128_$r.log 2> gpurun_out/ak_k128_$r.err || exit $?
  XCP_TN_XCD_ALIGN=1 timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 > gpurun_out/ak_xal_$r.log 2> gpurun_out/ak_xal_$r.err || exit $?
done
