"""Two ranks on the real kernels ("Parity at G>1"): XceptionLSTMV(128) B2T4 299^2,
unfrozen, fp32, each rank one shard of the clip batch through ``GradBuckets(module=model)`` -- the
engine's gradient sink, the bucket all-reduces launched from inside the backbone backward, the
1/world scaling and the rank-0 buffer broadcast -- against single-process runs of the two shards
(the reference's nn.DataParallel of train_audio.py:16-18 computes the same mean of per-shard
gradients, with BatchNorm statistics per shard: the reference has no SyncBN).

The ranks share cuda:0 through gloo (the one-GPU box; the measured configuration is RCCL, one GPU
per rank: ``bench.py --gpus N``).  Gloo all-reduces the device tensors through host memory; the
bucketing, overlap and scaling code under test is the same for both backends."""
import os

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp
import torch.nn as nn

pytestmark = pytest.mark.gpu

B_SHARD, T, S = 2, 4, 299


def _shard(rank):
    g = torch.Generator().manual_seed(1234 + rank)
    x = torch.rand((B_SHARD, T, 3, S, S), generator=g)
    y = torch.tensor([[float(rank % 2)], [1.0 - rank % 2]])
    return x, y


def _model(dev):
    from Models.XceptionLSTMV import XceptionLSTMV
    torch.manual_seed(0)
    m = XceptionLSTMV(128, pretrained=False)
    for p in m.feature_extractor.parameters():
        p.requires_grad = True
    m = m.to(dev).train()
    m.fc_layers.eval()   # dropout off (SURVEY §7 "Parity under randomness")
    return m


def _worker(rank, world, port, out):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import sys
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    for p in (os.path.join(repo, "multimodal-deepfake-detection_amd"), repo):
        if p not in sys.path:
            sys.path.insert(0, p)
    import xcp
    from xcp import ddp
    dist.init_process_group("gloo", rank=rank, world_size=world)
    dev = torch.device("cuda:0")
    xcp.load_library()
    m = _model(dev)
    params = list(m.parameters())
    gb = ddp.GradBuckets(params, world=world, module=m, bucket_bytes=8 << 20)
    x, y = _shard(rank)
    x, y = x.to(dev), y.to(dev)
    launched = []
    real = ddp.GradBuckets._launch

    def logged(self, bi):
        launched.append(bi)
        return real(self, bi)

    ddp.GradBuckets._launch = logged
    gb.zero()
    ddp.broadcast_buffers(m, use_streams=True)   # the stream form RCCL takes by default (gloo: the sync form)
    with xcp.precision("fp32"):
        loss = nn.BCELoss()(m(m.extract_features(x, dev)), y)
        loss.backward()
    n_during = len(launched)
    gb.allreduce()
    torch.cuda.synchronize()
    grads = {n: p.grad.detach().cpu().clone() for n, p in m.named_parameters()}
    own_bufs = {n: b.detach().cpu().clone() for n, b in m.named_buffers() if b.is_floating_point()}
    ddp.broadcast_buffers(m, use_streams=True)   # the next step's forward starts from rank 0's buffers
    torch.cuda.synchronize()
    bufs = {n: b.detach().cpu().clone() for n, b in m.named_buffers() if b.is_floating_point()}
    out[rank] = {"grads": grads, "bufs": bufs, "own_bufs": own_bufs, "loss": loss.item(),
                 "during": n_during, "buckets": len(gb.buckets)}
    dist.barrier()
    dist.destroy_process_group()


def test_two_rank_gradients_equal_mean_of_shards(gpu):
    import xcp
    world, port = 2, 29700 + os.getpid() % 1000
    ctx = mp.get_context("spawn")
    mgr = ctx.Manager()
    out = mgr.dict()
    mp.start_processes(_worker, args=(world, port, out), nprocs=world, join=True, start_method="spawn")
    # single-process runs of each shard (default autograd gradient delivery, no sink)
    ref_grads, ref_bufs = [], []
    for rank in range(world):
        m = _model(gpu)
        x, y = _shard(rank)
        with xcp.precision("fp32"):
            nn.BCELoss()(m(m.extract_features(x.to(gpu), gpu)), y.to(gpu)).backward()
        torch.cuda.synchronize()
        ref_grads.append({n: p.grad.detach().cpu() for n, p in m.named_parameters()})
        ref_bufs.append({n: b.detach().cpu() for n, b in m.named_buffers() if b.is_floating_point()})
    r0, r1 = out[0], out[1]
    assert r0["buckets"] > 4
    # the backbone's buckets are launched from inside its backward (all but the stem's)
    assert r0["during"] >= r0["buckets"] - 2, (r0["during"], r0["buckets"])
    worst = 0.0
    for n in ref_grads[0]:
        mean = 0.5 * (ref_grads[0][n].double() + ref_grads[1][n].double())
        for r in (r0, r1):
            got = r["grads"][n].double()
            err = float((got - mean).norm() / max(mean.norm(), 1e-30))
            worst = max(worst, err)
            assert err < 1e-5, (n, err)
    print(f"\nworst rank-vs-mean-of-shards gradient rel err: {worst:.2e}")
    # each rank's BatchNorm buffers come from its own shard (per-rank BN, no SyncBN) ...
    for rank, r in enumerate((r0, r1)):
        for n, b in ref_bufs[rank].items():
            np.testing.assert_allclose(r["own_bufs"][n].numpy(), b.numpy(), rtol=1e-5, atol=1e-6, err_msg=n)
    # ... and after the broadcast every rank holds rank 0's
    for n, b in r0["own_bufs"].items():
        assert torch.equal(r1["bufs"][n], b), n
        assert torch.equal(r0["bufs"][n], b), n
