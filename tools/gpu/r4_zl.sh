# Round 4 (zl): depthwise forward staged-tile size (FWD_MAXPX 512 default vs 256 / 1024, variant libraries):
# kernel times + output fingerprints at the step's shapes (tools/kbench.py dwshapes), in-step A/B, 3 rounds
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for v in base 256 1024; do
  if [ $v = base ]; then E="XCP_NONE=1"; else E="XCP_LIB_PATH=$PWD/tools/exp/dwpx$v/libxcp.so"; fi
  echo "== $v" >> gpurun_out/zl_kb.log
  env $E timeout -k 10 200 python -u tools/kbench.py dwshapes >> gpurun_out/zl_kb.log 2>&1 || exit $?
done
Q="--cpu-baseline off --mode unfrozen --small-batch 0 --measured-peaks off --diag off --no-kernel-timing"
for r in 1 2 3; do
  for v in base 256 1024; do
    if [ $v = base ]; then E="XCP_NONE=1"; else E="XCP_LIB_PATH=$PWD/tools/exp/dwpx$v/libxcp.so"; fi
    env $E timeout -k 10 240 python bench.py $Q > gpurun_out/zl_${v}_${r}.json 2>> gpurun_out/zl.err || exit $?
    echo "$v $(cat gpurun_out/zl_${v}_${r}.json)" >> gpurun_out/zl_step.log
  done
done
