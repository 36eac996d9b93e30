# GPU: LDS-DMA vs register-load fill bandwidth microbenchmark (tools/exp_ldsbw.*).
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 200 python -u tools/exp_ldsbw.py run > gpurun_out/r2_ldsbw.log 2>&1
