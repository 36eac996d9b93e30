# GPU: stem/block1 fusion -- kernel + model parity tests (fused, and the model tests again with
# XCP_STEM_FUSED=0), then bench A/B of the switch (on, off, on).
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 200 python -u -m pytest -x -q --timeout 150 --timeout-method thread tests/test_gpu_kernels.py -k "dw or bn_" > gpurun_out/stem_k.log 2>&1 || exit $?
timeout -k 10 300 python -u -m pytest -x -q --timeout 250 --timeout-method thread tests/test_gpu_model.py tests/test_gpu_train_step.py > gpurun_out/stem_m.log 2>&1 || exit $?
bash tools/gpu/r2_envab.sh XCP_STEM_FUSED
