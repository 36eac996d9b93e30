# Round 3 record (fourth, HEAD after the entry-flow GEMM tile rule): full -m gpu suite, smoke(), default
# bench (CPU baseline), then a HEAD kernel trace of the headline step (short: the pool had no free box for
# most of the session)
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -rf -p no:cacheprovider > gpurun_out/h_t.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/h_t.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 170 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/h_smoke.log 2>&1 || exit $?
timeout -k 10 600 python bench.py > gpurun_out/h_b.json 2> gpurun_out/h_b.err || exit $?
B="python bench.py --cpu-baseline off --mode unfrozen --steps 5 --warmup 2 --small-batch 0 --measured-peaks off --diag off"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_r3h -o kt -- $B > gpurun_out/h_prof.log 2>&1 || exit $?
