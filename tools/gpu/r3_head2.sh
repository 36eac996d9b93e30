# Round 3 HEAD record (after the 16-B aligned gradient views): op-level PMC traffic of the two
# roofline ops, default bench, then the HEAD profiles of the headline step
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
bash tools/gpu/r3_pmc_ops.sh || exit $?
timeout -k 10 600 python bench.py > gpurun_out/h2_b.json 2> gpurun_out/h2_b.err || exit $?
bash tools/gpu/r3_profile.sh > gpurun_out/h2_prof.log 2>&1
