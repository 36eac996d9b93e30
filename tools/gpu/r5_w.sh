# Round 5 (w): buffer-resource addressing (scalar row bases, 32-bit lane offsets) in the fused unit forward's
# row loads, the fused unit backward's tile loads / dD stores and the depthwise backward's LDS-DMA staging:
# GPU suite, kernel A/Bs (dw_ab, sep_bench, kbench unitbwd), in-step A/B base (HEAD) vs new, 3 rounds
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
T="python -u -m pytest -p no:cacheprovider --timeout 200 --timeout-method thread -rf"
timeout -k 10 400 $T -x -q -m gpu tests > gpurun_out/w_suite.log 2>&1 || exit $?
timeout -k 10 300 python -u tools/dw_ab.py run > gpurun_out/w_dwab.log 2>&1 || exit $?
for r in 1 2; do
  XCP_LIB_PATH=probe/base/libxcp.so timeout -k 10 200 python -u tools/sep_bench.py 10 > gpurun_out/w_sep_base_$r.log 2>&1 || exit $?
  timeout -k 10 200 python -u tools/sep_bench.py 10 > gpurun_out/w_sep_new_$r.log 2>&1 || exit $?
  XCP_LIB_PATH=probe/base/libxcp.so timeout -k 10 200 python -u tools/kbench.py unitbwd > gpurun_out/w_ub_base_$r.log 2>&1 || exit $?
  timeout -k 10 200 python -u tools/kbench.py unitbwd > gpurun_out/w_ub_new_$r.log 2>&1 || exit $?
done
for r in 1 2 3; do
  XCP_LIB_PATH=probe/base/libxcp.so timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 > gpurun_out/w_base_$r.log 2> gpurun_out/w_base_$r.err || exit $?
  timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 > gpurun_out/w_new_$r.log 2> gpurun_out/w_new_$r.err || exit $?
done
