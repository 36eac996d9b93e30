# Round 3: bench after the allocator fix (no record_stream on the backward side stream), then the GPU suite.
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 --cpu-baseline off > gpurun_out/r3_b3.json 2> gpurun_out/r3_b3.err || exit $?
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r3_t2.log 2>&1
echo "pytest rc=$?" >> gpurun_out/r3_t2.log
