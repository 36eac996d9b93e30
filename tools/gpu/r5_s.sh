# Round 5 (s): depthwise backward with one LDS object (rings + output staging) and asm staging reads (no
# vmcnt(0) drain of the look-ahead DMA in the plain-read form): dw tests, kernel A/B at the step's shapes,
# in-step A/B base (HEAD) / new / new with plain ring reads everywhere (XCP_DW_BWD_ASM=0), 3 rounds
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
T="python -u -m pytest -p no:cacheprovider --timeout 200 --timeout-method thread -rf"
timeout -k 10 300 $T -x -q tests/test_gpu_kernels.py -k "dw" > gpurun_out/s_dwtests.log 2>&1 || exit $?
timeout -k 10 300 python -u tools/dw_ab.py run > gpurun_out/s_dwab.log 2>&1 || exit $?
for r in 1 2 3; do
  XCP_LIB_PATH=probe/base/libxcp.so timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 > gpurun_out/s_base_$r.log 2> gpurun_out/s_base_$r.err || exit $?
  timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 > gpurun_out/s_new_$r.log 2> gpurun_out/s_new_$r.err || exit $?
  XCP_DW_BWD_ASM=0 timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 > gpurun_out/s_plain_$r.log 2> gpurun_out/s_plain_$r.err || exit $?
done
