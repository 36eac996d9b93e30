# GPU: NT GEMM epilogue with non-temporal stores (tools/exp/nt) vs the current library:
# kbench gemm (+ hipBLASLt at the same shapes), then bench A/B in one run.
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 200 python -u tools/kbench.py gemm blas > gpurun_out/nt_k_cur.log 2>&1 || exit $?
cp multimodal-deepfake-detection_amd/xcp/libxcp.so /tmp/libxcp_cur.so
cp tools/exp/nt/libxcp.so multimodal-deepfake-detection_amd/xcp/libxcp.so
timeout -k 10 200 python -u tools/kbench.py gemm > gpurun_out/nt_k_nt.log 2>&1 || exit $?
timeout -k 10 170 python -u bench.py --steps 20 --warmup 5 --cpu-baseline off > gpurun_out/nt_b_nt.json 2> gpurun_out/nt_b_nt.err || exit $?
cp /tmp/libxcp_cur.so multimodal-deepfake-detection_amd/xcp/libxcp.so
timeout -k 10 170 python -u bench.py --steps 20 --warmup 5 --cpu-baseline off > gpurun_out/nt_b_cur.json 2> gpurun_out/nt_b_cur.err
