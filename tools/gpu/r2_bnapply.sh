# GPU: BN-backward apply rows-per-thread A/B (current build: 4; tools/exp/rpt{1,2,8}) -- kbench
# bnapply per library, then the headline bench on the current build, after the BN parity tests.
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
LIB=multimodal-deepfake-detection_amd/xcp/libxcp.so
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -v --timeout 120 --timeout-method thread -m gpu \
  -k "bn or tail or unit" > gpurun_out/ba_tests.log 2>&1 || exit $?
timeout -k 10 120 python -u tools/kbench.py bnapply > gpurun_out/ba_rpt4a.txt 2>&1 || exit $?
cp $LIB /tmp/libxcp_cur.so
rc=0
for r in 1 2 8; do
  cp tools/exp/rpt$r/libxcp.so $LIB
  timeout -k 10 120 python -u tools/kbench.py bnapply > gpurun_out/ba_rpt$r.txt 2>&1 || { rc=$?; break; }
done
cp /tmp/libxcp_cur.so $LIB
[ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -u tools/kbench.py bnapply > gpurun_out/ba_rpt4b.txt 2>&1 || exit $?
timeout -k 10 170 python -u bench.py --steps 20 --warmup 5 --cpu-baseline off --measured-peaks off \
  > gpurun_out/ba_bench.json 2> gpurun_out/ba_bench.err
