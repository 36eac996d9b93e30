# GPU: bench A/B of one environment variable's values in one run.
# usage: bash tools/gpu/r2_envab2.sh VAR v1 v2 ...   (runs default, VAR=v1, VAR=v2, ..., default)
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
B="python -u bench.py --steps 20 --warmup 5 --cpu-baseline off"
var="$1"; shift
timeout -k 10 170 $B > gpurun_out/ev_def1.json 2> gpurun_out/ev_def1.err || exit $?
for v in "$@"; do
  env "$var=$v" timeout -k 10 170 $B > gpurun_out/ev_$v.json 2> gpurun_out/ev_$v.err || exit $?
done
timeout -k 10 170 $B > gpurun_out/ev_def2.json 2> gpurun_out/ev_def2.err
