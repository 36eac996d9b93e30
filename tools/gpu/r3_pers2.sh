# Round 3: persistent NT as the automatic choice -- GEMM tests, A/B, bench (default) vs bench XCP_NT_ONESHOT=1.
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -k "gemm or persistent or reduce_batch or unit" > gpurun_out/r3_pt2.log 2>&1 || exit $?
timeout -k 10 300 python -u tools/gemm_ab.py 5 > gpurun_out/r3_ab3.log 2>&1 || exit $?
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --cpu-baseline off --measured-peaks off > gpurun_out/r3_b5.json 2> gpurun_out/r3_b5.err || exit $?
XCP_NT_ONESHOT=1 timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --cpu-baseline off --measured-peaks off > gpurun_out/r3_b6.json 2> gpurun_out/r3_b6.err || exit $?
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --cpu-baseline off --measured-peaks off > gpurun_out/r3_b7.json 2> gpurun_out/r3_b7.err || exit $?
XCP_BF16_RECORD=1 timeout -k 10 900 python -u -m pytest tests -m gpu -q -s --timeout 300 --timeout-method thread -p no:cacheprovider -k "bf16 or block_module or backbone64 or lstma or frame_step or bench_size" > gpurun_out/r3_rec.log 2>&1
echo "pytest rc=$?" >> gpurun_out/r3_rec.log
