# Round 5 (ab): persistent NT GEMM with a dynamic tile queue (XCP_NT_DYNQ, default on) vs the static walk:
# GPU suite, in-step A/B (same library, env toggle), 3 rounds, and the kernel trace of each for the NT times
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
T="python -u -m pytest -p no:cacheprovider --timeout 200 --timeout-method thread -rf"
timeout -k 10 400 $T -x -q -m gpu tests > gpurun_out/ab_suite.log 2>&1 || exit $?
for r in 1 2 3; do
  XCP_NT_DYNQ=0 timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 > gpurun_out/ab_off_$r.log 2> gpurun_out/ab_off_$r.err || exit $?
  XCP_NT_DYNQ=1 timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 > gpurun_out/ab_on_$r.log 2> gpurun_out/ab_on_$r.err || exit $?
done
B="python -u bench.py --cpu-baseline off --mode unfrozen --steps 5 --warmup 2 --small-batch 0 --measured-peaks off --diag off --no-kernel-timing"
XCP_NT_DYNQ=0 timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/ab_prof_off -o kt -- $B > gpurun_out/ab_prof_off.log 2>&1 || exit $?
XCP_NT_DYNQ=1 timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/ab_prof_on -o kt -- $B > gpurun_out/ab_prof_on.log 2>&1 || exit $?
python tools/prof_summary.py gpurun_out/ab_prof_off 40 > gpurun_out/ab_kernels_off.txt 2>&1
python tools/prof_summary.py gpurun_out/ab_prof_on 40 > gpurun_out/ab_kernels_on.txt 2>&1
find gpurun_out/ab_prof_off gpurun_out/ab_prof_on -name "*kernel_trace.csv" -delete
