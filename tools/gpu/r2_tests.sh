# GPU: the full -m gpu suite only.
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -rf -s -p no:cacheprovider > gpurun_out/r2_t.log 2>&1
rc=$?
echo "pytest rc=$rc" >> gpurun_out/r2_t.log
exit $rc
