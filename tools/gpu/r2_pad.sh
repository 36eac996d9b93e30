# GPU: padded 728-channel pitch -- kernel + model parity tests, then bench A/B (XCP_PAD_728 on / off / on).
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 170 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -k "bn_ or reduce_slabs or unit_bwd or tail" > gpurun_out/pad_tests.log 2>&1 || exit $?
timeout -k 10 175 python -u -m pytest -x -q --timeout 170 --timeout-method thread tests/test_gpu_model.py tests/test_gpu_modules.py > gpurun_out/pad_model.log 2>&1 || exit $?
bash tools/gpu/r2_envab.sh XCP_PAD_728
