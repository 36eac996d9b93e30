# Round 3 record (fourth, HEAD after the entry-flow GEMM tile rule): full -m gpu suite, smoke(), default
# bench (CPU baseline), the 2-rank gloo path, C4 / C2 lines, then HEAD profiles (kernel trace + FETCH / WRITE
# passes) of the headline step
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -rf -p no:cacheprovider > gpurun_out/h_t.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/h_t.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 170 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/h_smoke.log 2>&1 || exit $?
timeout -k 10 600 python bench.py > gpurun_out/h_b.json 2> gpurun_out/h_b.err || exit $?
XCP_BENCH_BACKEND=gloo timeout -k 10 300 python bench.py --gpus 2 --steps 3 --warmup 1 --cpu-baseline off --small-batch 0 --measured-peaks off --no-kernel-timing > gpurun_out/h_g2.json 2> gpurun_out/h_g2.err || exit $?
timeout -k 10 170 python bench.py --model lstma --cpu-baseline off > gpurun_out/h_lstma.json 2> gpurun_out/h_lstma.err || exit $?
timeout -k 10 170 python bench.py --model xception --batch 64 --cpu-baseline off > gpurun_out/h_c2.json 2> gpurun_out/h_c2.err || exit $?
B="python bench.py --cpu-baseline off --mode unfrozen --steps 5 --warmup 2 --small-batch 0 --measured-peaks off --diag off"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_r3h -o kt -- $B > gpurun_out/h_prof.log 2>&1 || exit $?
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmch_fetch -o p -- $B --no-kernel-timing > gpurun_out/h_pmc_f.log 2>&1 || exit $?
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmch_write -o p -- $B --no-kernel-timing > gpurun_out/h_pmc_w.log 2>&1 || exit $?
