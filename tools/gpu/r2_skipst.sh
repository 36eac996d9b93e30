# GPU: skip-branch stream -- model / step / module / DDP-sink parity tests, then bench A/B of
# XCP_SKIP_STREAM (on, off, on).
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_model.py tests/test_gpu_train_step.py tests/test_gpu_modules.py tests/test_auface.py -m gpu > gpurun_out/skst_m.log 2>&1 || exit $?
bash tools/gpu/r2_envab.sh XCP_SKIP_STREAM
