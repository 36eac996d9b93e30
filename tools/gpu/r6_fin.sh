# Round 6: stem tail -- conv2 weight gradient shifted form (default) + BN1's finalize in 4-wave workgroups beside it
# (XCP_STEM_FIN_NARROW, default on).  Tests, kernel trace of the step, then A/B against the round-6 v4 stem
# (XCP_CONV3_WGRAD=0 XCP_STEM_FIN_NARROW=0), order rotated per repetition against box drift
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -k "conv3x3 or finalize_narrow or bn_padded" > gpurun_out/fin_tests.txt 2>&1 || exit $?
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_train_step.py tests/test_gpu_model.py > gpurun_out/fin_tests2.txt 2>&1 || exit $?
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_fin -o kt -- python -u bench.py --steps 5 --warmup 2 --cpu-baseline off --measured-peaks off --diag off > gpurun_out/fin_prof.log 2>&1 || exit $?
A="XCP_STEM_FIN_NARROW=1"; B="XCP_STEM_FIN_NARROW=0"; C="XCP_CONV3_WGRAD=0 XCP_STEM_FIN_NARROW=0"
for order in "A B C" "B C A" "C A B" "A C B"; do
for k in $order; do
  v=${!k}
  echo "== $v" >> gpurun_out/fin_ab.txt
  env $v timeout -k 10 200 python bench.py --cpu-baseline off --steps 20 --warmup 5 --measured-peaks off --diag off > gpurun_out/fin_one.json 2>> gpurun_out/fin_ab.err || exit $?
  grep '^{' gpurun_out/fin_one.json | python -c "import sys,json; d=json.loads(sys.stdin.read().splitlines()[-1]); print(d['value'], d['ms_per_step'])" >> gpurun_out/fin_ab.txt || exit $?
done; done
