# GPU: round-end record -- full -m gpu suite, smoke(), default bench (with CPU baseline), the
# multi-rank path (2 ranks sharing the GPU through the gloo test switch), and the C4 / C2 lines.
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -rf -p no:cacheprovider > gpurun_out/fin_t.log 2>&1
rc=$?
echo "pytest rc=$rc" >> gpurun_out/fin_t.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 170 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/fin_smoke.log 2>&1 || exit $?
timeout -k 10 600 python bench.py > gpurun_out/fin_b.json 2> gpurun_out/fin_b.err || exit $?
XCP_BENCH_BACKEND=gloo timeout -k 10 300 python bench.py --gpus 2 --steps 3 --warmup 1 --cpu-baseline off --small-batch 0 --measured-peaks off --no-kernel-timing > gpurun_out/fin_g2.json 2> gpurun_out/fin_g2.err || exit $?
timeout -k 10 170 python bench.py --model lstma --cpu-baseline off > gpurun_out/fin_lstma.json 2> gpurun_out/fin_lstma.err || exit $?
timeout -k 10 170 python bench.py --model xception --batch 64 --cpu-baseline off > gpurun_out/fin_c2.json 2> gpurun_out/fin_c2.err
