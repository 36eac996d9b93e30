# Round 4 (a): entry-flow GEMM kernel tests vs fp64, the bf16 model tests with the autocast-ensemble
# bound (record mode: every error and bound printed), the B4T16 bf16 step under the old tile rule,
# then the full -m gpu suite
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
T="python -u -m pytest -p no:cacheprovider --timeout 300 --timeout-method thread -rf"
timeout -k 10 300 $T tests/test_gpu_kernels.py -x -v -k "entry_flow or nt256_stats" > gpurun_out/a_kern.log 2>&1 || exit $?
XCP_BF16_RECORD=1 timeout -k 10 600 $T tests/test_gpu_model.py -s -v -k "bf16" > gpurun_out/a_rec.log 2>&1 || exit $?
XCP_NT_BIG_N256=0 XCP_BF16_RECORD=1 timeout -k 10 300 $T tests/test_gpu_model.py -s -v -k "bench_size and bf16 and b4t16" > gpurun_out/a_rec_n256off.log 2>&1 || exit $?
timeout -k 10 900 $T tests -m gpu -q > gpurun_out/a_suite.log 2>&1
echo "suite rc=$?" >> gpurun_out/a_suite.log
timeout -k 10 300 python -u tools/step_ablation.py --rounds 3 gemm_tn gemm_nt:728fwd gemm_nt:728dgrad gemm_nt:dgrad dw_bwd dw_fwd bn_bwd_apply colreduce_multi bn_bwd_reduce unit_bwd gemm_tn+colreduce_multi > gpurun_out/a_ablation.log 2>&1
