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


def test_pinned_reader_host_side(tmp_path):
    """PinnedClipReader's host half: FaceDataset's file order, labels and batching; each batch's
    uint8 frames [B, Tmax, H, W, 3] match collate_fn's padded fp32 clips x 255 on every valid
    frame; the host buffer is reused (and grown) across batches; mismatched frame sizes raise."""
    from Dataset.video_dataloader import PinnedClipReader
    rs = np.random.RandomState(4)
    for i, t in enumerate((4, 7, 2, 5, 3)):
        np.save(tmp_path / f"{'real' if i % 2 else 'fake'}_{i}.npy", rs.randint(0, 256, (t, 6, 8, 3), dtype=np.uint8))
    r = PinnedClipReader(str(tmp_path), 2, "cpu")
    assert len(r) == 3 and len(PinnedClipReader(str(tmp_path), 2, "cpu", drop_last=True)) == 2
    ref = list(get_face_dataloader(str(tmp_path), batch_size=2))
    buf = None
    for paths, (clips, labels) in zip(r.batches(), ref):
        buf, frames, lab, ln = PinnedClipReader.read_batch(paths, buf)
        assert frames.shape == (len(paths), int(ln.max()), 6, 8, 3)
        assert torch.equal(lab, labels)
        for i, t in enumerate(ln.tolist()):
            host = frames[i, :t].to(torch.float32).permute(0, 3, 1, 2) / 255.0
            assert torch.equal(host, clips[i, :t]) and float(clips[i, t:].abs().sum()) == 0.0
    sh = PinnedClipReader(str(tmp_path), 2, "cpu", shuffle=True, seed=1)
    assert sorted(sum(sh.batches(), [])) == r.files
    np.save(tmp_path / "fake_odd.npy", np.zeros((2, 5, 8, 3), np.uint8))
    with pytest.raises(ValueError):
        PinnedClipReader.read_batch([str(tmp_path / "fake_odd.npy"), r.files[0]])


@pytest.mark.gpu
@pytest.mark.parametrize("size,dtype,cl", [(None, torch.float32, False), ((299, 299), torch.float32, False),
                                           ((299, 299), torch.bfloat16, True), ((17, 40), torch.bfloat16, False),
                                           (None, torch.bfloat16, True)])
def test_frames_prep_vs_torch(size, dtype, cl):
    """xcp_frames_prep against torch on the CPU: x / 255 (bit-exact without resize), then
    F.interpolate(bilinear, align_corners=False) to the requested size (fp32 within 2e-6 of
    values in [0, 1]: ATen's vectorised CPU kernel forms the weights and sums in another
    order), bf16 = the fp32 result rounded (at most 1 bf16 ulp apart), channels_last
    storage, padding frames zero."""
    import torch.nn.functional as F
    from xcp import ops
    g = torch.Generator().manual_seed(5)
    B, T, H, W = 3, 4, 24, 20
    u8 = torch.randint(0, 256, (B, T, H, W, 3), generator=g, dtype=torch.uint8)
    lengths = torch.tensor([4, 1, 3], dtype=torch.int32)
    dev = torch.device("cuda:0")
    out = ops.frames_prep(u8.to(dev), lengths.to(dev), size, dtype, cl)
    torch.cuda.synchronize()
    OH, OW = size or (H, W)
    assert out.shape == (B, T, 3, OH, OW) and out.dtype == dtype
    assert out.permute(0, 1, 3, 4, 2).is_contiguous() if cl else out.is_contiguous()   # [B,T,OH,OW,3] storage
    x = u8.to(torch.float32).permute(0, 1, 4, 2, 3) / 255.0
    want = x if size is None else F.interpolate(x.reshape(B * T, 3, H, W), size=size, mode="bilinear",
                                                 align_corners=False).reshape(B, T, 3, OH, OW)
    for b, t in enumerate(lengths.tolist()):
        want[b, t:] = 0
    got = out.float().cpu()
    if dtype == torch.float32:
        if size is None:
            assert torch.equal(got, want)
        else:
            torch.testing.assert_close(got, want, rtol=1e-6, atol=2e-6)
    else:
        torch.testing.assert_close(got, want.to(torch.bfloat16).float(), rtol=2 ** -7, atol=1e-6)


@pytest.mark.gpu
def test_pinned_reader_gpu(tmp_path):
    """The full double-buffered path on the GPU (reader thread, pinned buffers, side-stream
    copy, frames_prep) equals the reference loader batch by batch."""
    from Dataset.video_dataloader import PinnedClipReader
    rs = np.random.RandomState(6)
    for i, t in enumerate((4, 7, 2, 5, 3)):
        np.save(tmp_path / f"{'real' if i % 2 else 'fake'}_{i}.npy", rs.randint(0, 256, (t, 16, 12, 3), dtype=np.uint8))
    ref = list(get_face_dataloader(str(tmp_path), batch_size=2))
    got = [(c.cpu(), lab.cpu(), ln.cpu()) for c, lab, ln in PinnedClipReader(str(tmp_path), 2, "cuda:0")]
    assert len(got) == len(ref)
    for (c, lab, ln), (rc, rl) in zip(got, ref):
        assert torch.equal(c, rc) and torch.equal(lab, rl)


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
