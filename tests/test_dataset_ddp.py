"""CPU tests: the reference-compatible data loaders and the one-process-per-GPU gradient
exchange (xcp.ddp) on a gloo world of 2."""
import os

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp
import torch.nn as nn

from Dataset.audio_dataloader import get_audio_dataloader
from Dataset.video_dataloader import get_face_dataloader


def test_face_loader(tmp_path):
    rs = np.random.RandomState(0)
    a = rs.randint(0, 256, (3, 8, 8, 3), dtype=np.uint8)
    b = rs.randint(0, 256, (5, 8, 8, 3), dtype=np.uint8)
    np.save(tmp_path / "real_a.npy", a)
    np.save(tmp_path / "fake_b.npy", b)
    clips, labels = next(iter(get_face_dataloader(str(tmp_path), batch_size=2)))
    assert clips.shape == (2, 5, 3, 8, 8) and clips.dtype == torch.float32
    # sorted order: fake_b, real_a
    assert labels.tolist() == [[1.0], [0.0]]
    np.testing.assert_allclose(clips[1, :3].numpy(), a.transpose(0, 3, 1, 2) / 255.0, rtol=1e-7)
    assert float(clips[1, 3:].abs().sum()) == 0.0   # zero padded


def test_face_loader_u8_host_side(tmp_path):
    """uint8 loader (GPU-expanded path): same files, order, labels and padding as
    get_face_dataloader; converting its batch on the host reproduces the fp32 batch."""
    from Dataset.video_dataloader import get_face_dataloader_u8
    rs = np.random.RandomState(2)
    a = rs.randint(0, 256, (3, 8, 12, 3), dtype=np.uint8)
    b = rs.randint(0, 256, (5, 8, 12, 3), dtype=np.uint8)
    np.save(tmp_path / "real_a.npy", a)
    np.save(tmp_path / "fake_b.npy", b)
    ref, ref_labels = next(iter(get_face_dataloader(str(tmp_path), batch_size=2)))
    u8, labels, lengths = next(iter(get_face_dataloader_u8(str(tmp_path), batch_size=2)))
    assert u8.dtype == torch.uint8 and u8.shape == (2, 5, 8, 12, 3)
    assert lengths.tolist() == [5, 3] and labels.tolist() == ref_labels.tolist()
    host = u8.to(torch.float32).permute(0, 1, 4, 2, 3) / 255.0
    assert torch.equal(host, ref)


@pytest.mark.gpu
def test_face_loader_u8_gpu_bitwise(tmp_path):
    """xcp_frames_u8_to_f32 (frames.hip) on the GPU equals the reference loader's fp32 batch
    bit for bit (x / 255, NCHW permute, zero padding of short clips)."""
    from Dataset.video_dataloader import clips_u8_to_device, get_face_dataloader_u8
    rs = np.random.RandomState(3)
    for i, t in enumerate((4, 7, 2)):
        np.save(tmp_path / f"{'real' if i == 1 else 'fake'}_{i}.npy", rs.randint(0, 256, (t, 20, 36, 3), dtype=np.uint8))
    ref, _ = next(iter(get_face_dataloader(str(tmp_path), batch_size=3)))
    batch = next(iter(get_face_dataloader_u8(str(tmp_path), batch_size=3)))
    clips, _ = clips_u8_to_device(batch, torch.device("cuda:0"))
    torch.cuda.synchronize()
    assert torch.equal(clips.cpu(), ref)


def test_audio_loader(tmp_path):
    m = np.random.RandomState(1).randn(120, 13).astype(np.float32)
    np.save(tmp_path / "real_x.npy", m)
    np.save(tmp_path / "fake_y.npy", m[:100])
    x, y = next(iter(get_audio_dataloader(str(tmp_path), batch_size=2)))
    assert x.shape == (2, 120, 3, 13)
    np.testing.assert_array_equal(x[1, :, 2].numpy(), m)
    assert float(x[0, 100:].abs().sum()) == 0.0


def _worker(rank, world, port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from xcp.ddp import GradBuckets, broadcast_buffers
    torch.manual_seed(0)
    model = nn.Sequential(nn.Linear(16, 32), nn.BatchNorm1d(32), nn.ReLU(), nn.Linear(32, 1))
    params = list(model.parameters())
    gb = GradBuckets(params, bucket_bytes=1024)
    assert len(gb.buckets) > 1
    if rank == 1:   # diverge buffers; broadcast must restore rank 0's
        model[1].running_mean.fill_(5.0)
    broadcast_buffers(model)
    rm = model[1].running_mean.clone()
    x = torch.randn(8, 16, generator=torch.Generator().manual_seed(100 + rank))
    for _ in range(2):   # two steps: hooks re-arm after zero()
        gb.zero()
        model(x).pow(2).mean().backward()
        gb.allreduce()
    out[rank] = {"grads": [p.grad.clone() for p in params], "rm": rm}
    dist.destroy_process_group()


def test_gradbuckets_allreduce_matches_mean_of_shards():
    world, port = 2, 29500 + os.getpid() % 1000
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_worker, args=(world, port, out), nprocs=world, join=True)
    # reference: per-shard gradients averaged (per-rank BN statistics, as DDP without SyncBN)
    ref = []
    for rank in range(world):
        torch.manual_seed(0)
        model = nn.Sequential(nn.Linear(16, 32), nn.BatchNorm1d(32), nn.ReLU(), nn.Linear(32, 1))
        x = torch.randn(8, 16, generator=torch.Generator().manual_seed(100 + rank))
        model(x).pow(2).mean().backward()
        ref.append([p.grad.clone() for p in model.parameters()])
    mean = [(a + b) / 2 for a, b in zip(*ref)]
    for rank in range(world):
        for g, r in zip(out[rank]["grads"], mean):
            torch.testing.assert_close(g, r, rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(out[0]["rm"], out[1]["rm"])
