# Round 4 (g): depthwise backward ring-read form chosen per frame height (kernel tests, tools/dw_ab.py
# against the plain-read library); weight-gradient splits whole per XCD (XCP_TN_XCD_ALIGN): bitwise
# test, kernel times and HBM traffic per variant (tools/tn_align.py), in-step A/B
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest -p no:cacheprovider --timeout 200 --timeout-method thread -rf tests/test_gpu_kernels.py -q \
  -k "ring_read_forms or row_bands or xcd_align_bitwise or gemm_tn or dw_fwd_bwd" > gpurun_out/g_tests.log 2>&1 || exit $?
timeout -k 10 300 python -u tools/dw_ab.py run > gpurun_out/g_dwab.log 2>&1 || exit $?
timeout -k 10 200 python -u tools/tn_align.py time > gpurun_out/g_tn.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/g_pmc_fetch -o p -- python tools/tn_align.py pmc > gpurun_out/g_pmc_f.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/g_pmc_write -o p -- python tools/tn_align.py pmc > gpurun_out/g_pmc_w.log 2>&1 || exit $?
python tools/pmc_traffic.py $(find gpurun_out/g_pmc_fetch -name "*counter_collection.csv" | head -1) $(find gpurun_out/g_pmc_write -name "*counter_collection.csv" | head -1) gpurun_out/g_tntraffic.json gemm_tn > gpurun_out/g_pmc.log 2>&1 || exit $?
Q="--cpu-baseline off --mode unfrozen --small-batch 0 --measured-peaks off --diag off --no-kernel-timing"
for r in 1 2; do
  for v in 0 1; do
    XCP_TN_XCD_ALIGN=$v timeout -k 10 200 python bench.py $Q > gpurun_out/g_step_${v}_${r}.json 2>> gpurun_out/g_step.err || exit $?
    echo "XCP_TN_XCD_ALIGN=$v $(cat gpurun_out/g_step_${v}_${r}.json)" >> gpurun_out/g_step.log
  done
done
