# Round 4 (zn): the stem conv2 weight gradient on fewer workgroups (XCP_CONV3_WGRAD_WGS: several (frame, band)
# jobs per workgroup, CUs left to the main stream's BN1 finalize and conv1 weight gradient): conv3x3 tests at the
# default grid and at a capped one, in-step A/B default / 192 / 128, 3 rounds
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest -p no:cacheprovider --timeout 150 --timeout-method thread -rf tests/test_gpu_kernels.py -q \
  -k "conv3x3 or conv2 or stem" > gpurun_out/zn_tests.log 2>&1 || exit $?
XCP_CONV3_WGRAD_WGS=37 timeout -k 10 300 python -u -m pytest -p no:cacheprovider --timeout 150 --timeout-method thread -rf tests/test_gpu_kernels.py -q \
  -k "conv3x3 or conv2 or stem" > gpurun_out/zn_tests37.log 2>&1 || exit $?
Q="--cpu-baseline off --mode unfrozen --small-batch 0 --measured-peaks off --diag off --no-kernel-timing"
for r in 1 2 3; do
  for v in 0 192 128; do
    XCP_CONV3_WGRAD_WGS=$v timeout -k 10 240 python bench.py $Q > gpurun_out/zn_${v}_${r}.json 2>> gpurun_out/zn.err || exit $?
    echo "$v $(cat gpurun_out/zn_${v}_${r}.json)" >> gpurun_out/zn_step.log
  done
done
