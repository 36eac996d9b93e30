# Round 4 (zb): the multi-rank bench path at HEAD, two ranks on the one GPU of the box over gloo
# (XCP_BENCH_BACKEND=gloo; the measured N > 1 configuration is RCCL, one GPU per rank -- the driver's)
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
XCP_BENCH_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29531 bench.py --gpus 2 --steps 3 --warmup 1 --cpu-baseline off \
  --small-batch 0 --measured-peaks off > gpurun_out/zb_bench2.json 2> gpurun_out/zb_bench2.err || exit $?
