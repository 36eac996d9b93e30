# Round 4 (m): bench-size bf16 test with 12 autocast draws (time), conv1-rescaled engine realizations
# (backbone64), conv3x3 two-workgroup forward (test, tools/conv3_ab.py), in-step A/B of the stem's
# conv2 weight-gradient launch point (XCP_STEM_WGRAD_EARLY) and of XCP_CONV3_FWD_2WG
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
( while true; do date >> gpurun_out/m_heartbeat.txt; sleep 50; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
timeout -k 10 400 python -u -m pytest -p no:cacheprovider --timeout 300 --timeout-method thread -rf -s -v tests/test_gpu_model.py \
  -k "b16t16 and bf16 or backbone64 and bf16" --durations=5 > gpurun_out/m_model.log 2>&1 || exit $?
timeout -k 10 200 python -u -m pytest -p no:cacheprovider --timeout 150 --timeout-method thread -rf tests/test_gpu_kernels.py -q \
  -k "conv3x3" > gpurun_out/m_tests.log 2>&1 || exit $?
timeout -k 10 200 python -u tools/conv3_ab.py > gpurun_out/m_conv3.log 2>&1 || exit $?
Q="--cpu-baseline off --mode unfrozen --small-batch 0 --measured-peaks off --diag off --no-kernel-timing"
for r in 1 2; do
  for v in 00 10 01; do
    XCP_STEM_WGRAD_EARLY=${v:0:1} XCP_CONV3_FWD_2WG=${v:1:1} timeout -k 10 200 python bench.py $Q > gpurun_out/m_step_${v}_${r}.json 2>> gpurun_out/m_step.err || exit $?
    echo "XCP_STEM_WGRAD_EARLY/CONV3_FWD_2WG=$v $(cat gpurun_out/m_step_${v}_${r}.json)" >> gpurun_out/m_step.log
  done
done
