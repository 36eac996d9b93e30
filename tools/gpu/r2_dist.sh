# GPU: the multi-rank bench path on a one-GPU box (2 ranks sharing cuda:0 over gloo; test
# only -- the measured configuration is RCCL, one GPU per rank): lstmv both modes, auface.
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0 XCP_BENCH_BACKEND=gloo
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 python bench.py --gpus 2 --batch 2 --frames 4 --steps 3 --warmup 1 --cpu-baseline off > gpurun_out/r2_dist_lstmv.json 2> gpurun_out/r2_dist_lstmv.err || exit $?
timeout -k 10 400 python bench.py --gpus 2 --model auface --batch 2 --frames 4 --steps 4 --warmup 4 > gpurun_out/r2_dist_auface.json 2> gpurun_out/r2_dist_auface.err
