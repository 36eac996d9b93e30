# Round 5 (z): depthwise backward calls with a strided-skip gradient (first units of blocks 2, 3, 12) on the
# one-row-look-ahead plain-read form (3 waves / SIMD) instead of the round-2 two-row form: dw tests, kernel A/B
# incl. the skip shapes, in-step A/B base (HEAD) / new / new with XCP_DW_BWD_SKIP4=0, 3 rounds
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
T="python -u -m pytest -p no:cacheprovider --timeout 200 --timeout-method thread -rf"
timeout -k 10 300 $T -x -q tests/test_gpu_kernels.py -k "dw" > gpurun_out/z_dwtests.log 2>&1 || exit $?
timeout -k 10 400 python -u tools/dw_ab.py run > gpurun_out/z_dwab.log 2>&1 || exit $?
for r in 1 2 3; do
  XCP_LIB_PATH=probe/base/libxcp.so timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 > gpurun_out/z_base_$r.log 2> gpurun_out/z_base_$r.err || exit $?
  timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 > gpurun_out/z_new_$r.log 2> gpurun_out/z_new_$r.err || exit $?
  XCP_DW_BWD_SKIP4=0 timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 > gpurun_out/z_off_$r.log 2> gpurun_out/z_off_$r.err || exit $?
done
