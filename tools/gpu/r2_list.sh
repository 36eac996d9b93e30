# GPU: list the PMC counters rocprofv3 offers on this device.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 120 rocprofv3 -L > gpurun_out/r2_counters.txt 2>&1
