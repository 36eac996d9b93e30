# Round 5 (f): folded vs partial-row BN finalizes on one model step (tools/fold_ab.py), then the C2 / C1
# frame-step tests under both settings
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u tools/fold_ab.py 8 299 > gpurun_out/f_ab.log 2>&1 || exit $?
timeout -k 10 300 python -u tools/fold_ab.py 64 299 >> gpurun_out/f_ab.log 2>&1 || exit $?
T="python -u -m pytest -p no:cacheprovider --timeout 200 --timeout-method thread -rf"
XCP_BN_FOLD=0 timeout -k 10 400 $T -q tests/test_gpu_model.py -k "frame_step and fp32" > gpurun_out/f_nofold.log 2>&1; echo "nofold rc $?" >> gpurun_out/f_ab.log
