# Round 3: HBM traffic per launch of the bench's two roofline ops at the step's shape (separate
# FETCH_SIZE / WRITE_SIZE passes over tools/kbench.py roof_ops) -> gpurun_out/optraffic.json
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmco_fetch -o p -- python tools/kbench.py roof_ops > gpurun_out/pmco_f.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmco_write -o p -- python tools/kbench.py roof_ops > gpurun_out/pmco_w.log 2>&1 || exit $?
python tools/pmc_traffic.py $(find gpurun_out/pmco_fetch -name "*counter_collection.csv" | head -1) $(find gpurun_out/pmco_write -name "*counter_collection.csv" | head -1) gpurun_out/optraffic.json > gpurun_out/pmco.log 2>&1
