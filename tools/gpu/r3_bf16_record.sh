# Round 3: measure every bf16 gradient-norm error above the 5e-2 contract (XCP_BF16_RECORD=1) over the GPU suite.
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
XCP_BF16_RECORD=1 timeout -k 10 900 python -u -m pytest tests -m gpu -q -s --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r3_rec.log 2>&1
echo "pytest rc=$?" >> gpurun_out/r3_rec.log
