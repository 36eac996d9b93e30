# Round 5 (j): depthwise forward walking frames last-to-first (XCP_DW_FWD_REV=1: the frames its producer wrote
# last are the ones still in the Infinity Cache) -- dw tests with it on, then in-step A/B (3 rounds, alternating,
# per-op timing on: roofline_dw.avg_launch_ms is the in-step launch time)
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
T="python -u -m pytest -p no:cacheprovider --timeout 200 --timeout-method thread -rf"
XCP_DW_FWD_REV=1 timeout -k 10 300 $T -q tests/test_gpu_kernels.py -k "dw_fwd" > gpurun_out/j_tests.log 2>&1 || exit $?
Q="--cpu-baseline off --mode unfrozen --small-batch 0 --measured-peaks off --diag off"
for r in 1 2 3; do
  for v in 1 0; do
    XCP_DW_FWD_REV=$v timeout -k 10 240 python bench.py $Q > gpurun_out/j_${v}_${r}.json 2>> gpurun_out/j.err || exit $?
    python -c "import json,sys; d=json.load(open('gpurun_out/j_${v}_${r}.json')); print('$v', d['value'], d['ms_per_step'], d['roofline_dw']['avg_launch_ms'], d['roofline']['avg_launch_ms'])" >> gpurun_out/j_step.log
  done
done
# 2-rank gloo path (two ranks sharing the GPU): buffer broadcast sync (gloo default now) vs stream form, bucket
# launches from the main stream
timeout -k 10 300 $T -q tests/test_gpu_ddp.py > gpurun_out/j_ddp.log 2>&1 || exit $?
G="python bench.py --gpus 2 --cpu-baseline off --mode unfrozen --steps 3 --warmup 1 --small-batch 0 --measured-peaks off --diag off --no-kernel-timing"
for cfg in "XCP_BCAST_STREAMS=0" "XCP_BCAST_STREAMS=1" "XCP_DDP_LAUNCH=main"; do
  env XCP_BENCH_BACKEND=gloo $cfg timeout -k 10 300 $G > gpurun_out/j_g2.json 2>> gpurun_out/j_g2.err || exit $?
  echo "$cfg $(python -c "import json; d=json.load(open('gpurun_out/j_g2.json')); print(d['value'], d['ms_per_step'])")" >> gpurun_out/j_g2.log
done
