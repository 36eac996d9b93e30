# GPU: rocprofv3 kernel trace + stats of the bench, and the two HBM-traffic PMC passes
# (FETCH_SIZE, WRITE_SIZE: separate runs) of the same command.
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
B="python bench.py --cpu-baseline off --mode unfrozen --steps 5 --warmup 2 --small-batch 0 --measured-peaks off"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_r2 -o kt -- $B > gpurun_out/r2_prof.log 2>&1 || exit $?
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_fetch -o p -- $B --no-kernel-timing > gpurun_out/r2_pmc_f.log 2>&1 || exit $?
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_write -o p -- $B --no-kernel-timing > gpurun_out/r2_pmc_w.log 2>&1 || exit $?
echo ok
