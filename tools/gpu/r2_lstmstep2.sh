# GPU: per-step LSTM kernels (bank-spread LDS reads): LSTM parity tests,
# rocprofv3 kernel traces (current vs tools/exp/lstmold), XceptionLSTMA line.
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_model.py -x -v --timeout 120 \
  --timeout-method thread -m gpu -k "lstm" > gpurun_out/ls2_tests.log 2>&1 || exit $?
bash tools/gpu/r2_lstmprof.sh || exit $?
timeout -k 10 170 python -u bench.py --model lstma --steps 30 --warmup 5 --cpu-baseline off --measured-peaks off \
  > gpurun_out/ls2_bench.json 2> gpurun_out/ls2_bench.err
