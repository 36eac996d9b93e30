# GPU: full -m gpu suite, smoke(), then the default bench (with its CPU baseline).
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -rf -p no:cacheprovider > gpurun_out/r2_t.log 2>&1
rc=$?
echo "pytest rc=$rc" >> gpurun_out/r2_t.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 170 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r2_smoke.log 2>&1 || exit $?
timeout -k 10 600 python bench.py > gpurun_out/r2_b.json 2> gpurun_out/r2_b.err
