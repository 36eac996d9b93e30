# GPU: fused unit-backward tests + micro-benchmark, then the model-level parity tests.
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 170 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -k "unit_bwd or reduce_slabs or dw_fwd_bwd or bn_forward" > gpurun_out/unit_tests.log 2>&1 || exit $?
timeout -k 10 170 python -u tools/kbench.py unitbwd > gpurun_out/unit_kb.log 2>&1 || exit $?
timeout -k 10 175 python -u -m pytest -x -q --timeout 170 --timeout-method thread tests/test_gpu_model.py > gpurun_out/unit_model.log 2>&1
