# Round 4 (q): the default bench line (as the driver runs it) against --diag off, interleaved x2
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for r in 1 2; do
  timeout -k 10 600 python bench.py > gpurun_out/q_default_${r}.json 2>> gpurun_out/q.err || exit $?
  echo "default $(tail -1 gpurun_out/q_default_${r}.json)" >> gpurun_out/q.log
  timeout -k 10 600 python bench.py --diag off --cpu-baseline off --measured-peaks off > gpurun_out/q_nodiag_${r}.json 2>> gpurun_out/q.err || exit $?
  echo "nodiag $(tail -1 gpurun_out/q_nodiag_${r}.json)" >> gpurun_out/q.log
done
