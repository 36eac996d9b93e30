# GPU: fusion-model tests, the C5 (auface) bench small then at its default size, and the C2 bench.
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 python -u -m pytest tests/test_auface.py tests/test_dataset_ddp.py -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r2_af_t.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/r2_af_t.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --model auface --batch 2 --frames 4 --steps 4 --warmup 4 > gpurun_out/r2_af_small.json 2> gpurun_out/r2_af_small.err || exit $?
timeout -k 10 400 python -u bench.py --model auface --steps 8 --warmup 4 > gpurun_out/r2_af.json 2> gpurun_out/r2_af.err || exit $?
timeout -k 10 300 python -u bench.py --model xception --batch 64 --steps 10 --warmup 3 > gpurun_out/r2_c2.json 2> gpurun_out/r2_c2.err
