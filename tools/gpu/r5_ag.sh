# Round 5 (ag): with the tile queue, the sparse last NT round (XCP_NT_SPARSE=0: every row on the persistent kernel)
# in-step A/B, 3 rounds
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for r in 1 2 3; do
  timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 > gpurun_out/ag_on_$r.log 2> gpurun_out/ag_on_$r.err || exit $?
  XCP_NT_SPARSE=0 timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 > gpurun_out/ag_off_$r.log 2> gpurun_out/ag_off_$r.err || exit $?
done
