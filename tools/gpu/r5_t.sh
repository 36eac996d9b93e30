# Round 5 (t): packed bf16 conversions (one v_cvt_pk_bf16_f32 per pair: pk_bf16) in the depthwise, fused unit
# forward, GEMM / conv2 epilogues and the conv2 activation; the depthwise forward's staging and stores on
# incremental 32-bit buffer offsets: GPU suite, depthwise backward kernel A/B, depthwise forward shapes
# (kbench dwshapes, fingerprints), fused forward A/B, in-step A/B base (HEAD) vs new, 3 rounds
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
T="python -u -m pytest -p no:cacheprovider --timeout 200 --timeout-method thread -rf"
timeout -k 10 400 $T -x -q -m gpu tests > gpurun_out/t_suite.log 2>&1 || exit $?
timeout -k 10 300 python -u tools/dw_ab.py run > gpurun_out/t_dwab.log 2>&1 || exit $?
for r in 1 2; do
  XCP_LIB_PATH=probe/base/libxcp.so timeout -k 10 200 python -u tools/kbench.py dwshapes > gpurun_out/t_dwf_base_$r.log 2>&1 || exit $?
  timeout -k 10 200 python -u tools/kbench.py dwshapes > gpurun_out/t_dwf_new_$r.log 2>&1 || exit $?
done
for r in 1 2; do
  XCP_LIB_PATH=probe/base/libxcp.so timeout -k 10 200 python -u tools/sep_bench.py 10 > gpurun_out/t_sep_base_$r.log 2>&1 || exit $?
  timeout -k 10 200 python -u tools/sep_bench.py 10 > gpurun_out/t_sep_new_$r.log 2>&1 || exit $?
done
for r in 1 2 3; do
  XCP_LIB_PATH=probe/base/libxcp.so timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 > gpurun_out/t_base_$r.log 2> gpurun_out/t_base_$r.err || exit $?
  timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 > gpurun_out/t_new_$r.log 2> gpurun_out/t_new_$r.err || exit $?
done
