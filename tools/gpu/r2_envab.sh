# GPU: bench A/B of one environment switch in one run (on, off, on).
# usage: bash tools/gpu/r2_envab.sh VAR   (runs with VAR unset, VAR=0, VAR unset)
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
B="python -u bench.py --steps 20 --warmup 5 --cpu-baseline off"
timeout -k 10 170 $B > gpurun_out/envab_on1.json 2> gpurun_out/envab_on1.err || exit $?
env "$1=0" timeout -k 10 170 $B > gpurun_out/envab_off.json 2> gpurun_out/envab_off.err || exit $?
timeout -k 10 170 $B > gpurun_out/envab_on2.json 2> gpurun_out/envab_on2.err
