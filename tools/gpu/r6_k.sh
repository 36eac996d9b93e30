# Round 6 (k): non-temporal stores on the other big streaming producers of the step, one variant each (linked by
# tools/build_variant.py): the depthwise forward / backward outputs (probe/dwnt), the BN-backward apply's dY (probe/bnnt);
# the lstmv step, interleaved, 2 rounds
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for r in 1 2; do
  timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --cpu-baseline off > gpurun_out/k_base_$r.log 2> gpurun_out/k_base_$r.err || exit $?
  XCP_LIB_PATH=probe/dwnt/libxcp.so timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --cpu-baseline off > gpurun_out/k_dwnt_$r.log 2> gpurun_out/k_dwnt_$r.err || exit $?
  XCP_LIB_PATH=probe/bnnt/libxcp.so timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --cpu-baseline off > gpurun_out/k_bnnt_$r.log 2> gpurun_out/k_bnnt_$r.err || exit $?
done
