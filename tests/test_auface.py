"""The build-defined AU + face fusion model (Models/AUFaceModel.py) and the train_au_face.py
harness (xcp/auface.py), BASELINE config C5.

The reference's AUFaceCrossDetector is absent from the snapshot, so there is no reference
output to pin: parity is between the HIP path and the oracle's functional restatement of
the same definition (oracle.auface_forward), and the oracle is pinned to the module
definition on the CPU (backbones through the oracle's Xception, which test_oracle_golden
pins to the reference).  Parity against the reference itself: unpinned.
"""
import copy

import numpy as np
import pytest
import torch
import torch.nn as nn

from oracle import xception_oracle as O


def seeded(shape, seed):
    return torch.rand(shape, generator=torch.Generator().manual_seed(seed), dtype=torch.float32)


def small_model(seed=0):
    from Models.AUFaceModel import AUFaceCrossDetector
    torch.manual_seed(seed)
    return AUFaceCrossDetector(num_aus=17, face_dim=512, au_dim=512, lstm_hidden=256)


def test_model_surface_and_oracle_matches_module_definition():
    """Constructor / forward contract of train_au_face.py:594, :656 and test_au_face.py:169, and
    oracle.auface_forward == the module composition (backbones and LSTM through the CPU
    restatements, everything else the modules themselves)."""
    m = small_model().train()
    sd = m.state_dict()
    assert any(k.startswith("face_backbone.block4.") for k in sd) and any(k.startswith("au_backbone.") for k in sd)
    assert "cross.in_proj_weight" in sd and "temporal.weight_hh_l0" in sd
    with pytest.raises(ValueError):
        m.au_tokens(torch.zeros(1, 18, 3, 8, 8))
    assert m.frames_first(torch.zeros(2, 3, 5, 8, 8)).shape == (2, 5, 3, 8, 8)
    with pytest.raises(ValueError):
        m.frames_first(torch.zeros(2, 5, 4, 8, 8))
    # CPU stand-ins for the GPU-only parts, fed the same parameters
    for name in ("face_backbone", "au_backbone"):
        bb = getattr(m, name)
        bb.forward = (lambda x, _p=name: O.backbone_forward(x, dict(m.named_parameters()) | dict(m.named_buffers()),
                                                              True, None, prefix=_p + "."))
    lstm = nn.LSTM(512, 256, batch_first=True)
    lstm.load_state_dict({k.split(".", 1)[1]: v for k, v in sd.items() if k.startswith("temporal.")})
    m.temporal.forward = lambda x: lstm(x)
    videos = seeded((2, 3, 3, 64, 64), 1)          # [B, 3, T, H, W] as the harness passes it
    aus = seeded((2, 4, 3, 64, 64), 2)
    mask = torch.tensor([[1., 1., 0., 1.], [0., 0., 0., 0.]])
    weight = torch.tensor([[1., .5, 1., .25], [1., 1., 1., 1.]])
    with torch.no_grad():
        got = m(videos, aus, au_mask=mask, au_weight=weight)
        want = O.auface_forward(videos.permute(0, 2, 1, 3, 4), aus, sd, mask, weight)
    assert got[0].shape == (2, 2) and got[1].shape == (2, 3, 512) and got[2].shape == (2, 4, 512)
    for a, b in zip(got, want):
        torch.testing.assert_close(a, b, rtol=1e-5, atol=1e-5)


def test_trainer_construction_and_checkpoint_cpu(tmp_path):
    """AUFaceTrainer wiring on the CPU (no compute): the LazyLinear embed head is materialised
    before averaging, AdamW / OneCycleLR / GradScaler are built as train_au_face.py:598-624,
    and the checkpoint of :751-756 loads back through load_state_dict_flexible strictly."""
    from xcp.auface import AUFaceTrainer, unpack_batch
    from xcp.checkpoint import load_state_dict_flexible
    m = small_model()
    tr = AUFaceTrainer(m, samples_per_cls=(300, 1700), use_amp=False)
    assert tr.embed_head[0].in_features == 1024 and tr.ema_model is not None
    assert len(tr.optimizer.param_groups[0]["params"]) == len(tr.params)
    assert tr.optimizer.param_groups[0]["lr"] == pytest.approx(1e-3 / 25)   # OneCycleLR initial lr
    np.testing.assert_allclose(tr.cbfocal.class_weights.numpy(), O.cb_class_weights([300, 1700]).numpy(), rtol=1e-6)
    ck = tr.state_dict(best_auc=0.5)
    torch.save(ck, tmp_path / "auface.pth")
    fresh = small_model(seed=1)
    missing, unexpected = load_state_dict_flexible(fresh, str(tmp_path / "auface.pth"), verbose=False)
    assert not missing and not unexpected
    for (k, a), b in zip(fresh.state_dict().items(), m.state_dict().values()):
        assert torch.equal(a, b), k
    assert len(unpack_batch((1, 2, 3))) == 5
    with pytest.raises(RuntimeError):
        unpack_batch((1, 2))


@pytest.mark.gpu
@pytest.mark.parametrize("T,A,S", [(3, 4, 64), (75, 17, 128)], ids=["small", "reference_shape"])
def test_auface_forward_backward_vs_oracle(gpu, T, A, S):
    """HIP path vs oracle.auface_forward in fp32: logits, both token streams, the harness loss
    (CB-focal on ArcFace(m=0.30) of the embed head, + 0.2 align + 0.1 temporal; embed head in
    eval so its dropout is off), and every parameter's gradient norm (test_gpu_model contract:
    1e-3, BatchNorm affine 5e-3).  ``reference_shape`` is train_au_face.py:563-570's own
    per-step shape: batch 2, 75 frames, 17 AUs, 128 x 128."""
    import xcp
    from xcp.auface import auface_losses
    from xcp.heads import ArcFaceHead, CBFocalLoss
    m = small_model().train()
    sd_cpu = {k: v.clone().requires_grad_(v.is_floating_point() and "running" not in k and "num_batches" not in k)
              for k, v in m.state_dict().items()}
    torch.manual_seed(3)
    embed = nn.Sequential(nn.Linear(1024, 256), nn.ReLU(), nn.Dropout(0.2), nn.Linear(256, 128)).eval()
    embed_cpu = copy.deepcopy(embed)
    torch.manual_seed(4)
    arc = ArcFaceHead(128, 2, s=30.0, m=0.30)
    w_cpu = arc.weight.detach().clone().requires_grad_(True)
    m, embed, arc = m.to(gpu), embed.to(gpu), arc.to(gpu)
    cb = CBFocalLoss([300, 1700]).to(gpu)
    videos = seeded((2, 3, T, S, S), 11)
    aus = seeded((2, A, 3, S, S), 12)
    if A == 4:
        mask = torch.tensor([[1., 1., 0., 1.], [1., 0., 1., 1.]])
        weight = torch.tensor([[1., .5, 1., .25], [1., 1., .75, 1.]])
    else:   # some AUs absent (mask 0) and uneven weights, as the dataset's per-AU detection gives
        g = torch.Generator().manual_seed(13)
        mask = (torch.rand(2, A, generator=g) > 0.25).float()
        weight = 0.25 + 0.75 * torch.rand(2, A, generator=g)
    labels = torch.tensor([0, 1])
    with xcp.precision("fp32"):
        logits, v_tok, au_tok = m(videos.to(gpu), aus.to(gpu), au_mask=mask.to(gpu), au_weight=weight.to(gpu))
        e = embed(torch.cat([v_tok.mean(1), au_tok.mean(1)], 1))
        loss = auface_losses(arc(e, labels.to(gpu)), labels.to(gpu), v_tok, au_tok, cb)[0]
        loss.backward()
    torch.cuda.synchronize()
    r_logits, r_v, r_au = O.auface_forward(videos.permute(0, 2, 1, 3, 4), aus, sd_cpu, mask, weight)
    r_e = embed_cpu(torch.cat([r_v.mean(1), r_au.mean(1)], 1))
    r_arc = O.arcface_logits(r_e, w_cpu, labels, 30.0, 0.30)
    r_pool_v, r_pool_a = r_v.mean(1), r_au.mean(1)
    r_loss = (O.cb_focal_loss(r_arc, labels, O.cb_class_weights([300, 1700])) + 0.2 * ((r_pool_v - r_pool_a) ** 2).mean()
              + 0.1 * 0.5 * ((r_v[:, 1:] - r_v[:, :-1]).pow(2).mean() + (r_au[:, 1:] - r_au[:, :-1]).pow(2).mean()))
    r_loss.backward()
    torch.testing.assert_close(logits.cpu(), r_logits.detach(), rtol=1e-4, atol=1e-4)
    torch.testing.assert_close(v_tok.cpu(), r_v.detach(), rtol=1e-4, atol=1e-5)
    torch.testing.assert_close(au_tok.cpu(), r_au.detach(), rtol=1e-4, atol=1e-5)
    np.testing.assert_allclose(loss.item(), r_loss.item(), rtol=1e-4)
    bad = []
    for n, p in m.named_parameters():
        want = sd_cpu[n].grad
        if want is None:
            assert p.grad is None or float(p.grad.abs().max()) == 0.0, n
            continue
        e_ = abs(p.grad.double().norm().item() - want.double().norm().item()) / max(want.double().norm().item(), 1e-12)
        if e_ > (5e-3 if p.dim() == 1 and "backbone" in n else 1e-3):
            bad.append((n, e_))
    assert not bad, bad[:5]
    e_ = abs(arc.weight.grad.double().norm().item() - w_cpu.grad.double().norm().item()) / w_cpu.grad.double().norm()
    assert e_ < 1e-3


@pytest.mark.gpu
def test_auface_trainer_accumulation_ema_eval(gpu):
    """Four micro-batches of the harness under autocast (bf16 backbones, GradScaler): finite
    losses, one optimizer step at the 4th, one AveragedModel update (n_averaged = 1; the
    averaged parameters then equal the model's), scheduler advanced, eval scores in [0, 1].
    (GradScaler starts at 2^8 here: at the default 2^16 the fp16 head gradients of a fresh
    model overflow and the scaler skips its first steps, as it would in the script.)"""
    from xcp.auface import AUFaceTrainer
    m = small_model().to(gpu)
    tr = AUFaceTrainer(m, samples_per_cls=(300, 1700), steps_per_epoch=8, init_scale=2.0 ** 8)
    tr.train()
    lr0 = tr.optimizer.param_groups[0]["lr"]
    before = [p.detach().clone() for p in m.parameters()]
    for i in range(4):
        batch = (seeded((2, 3, 3, 64, 64), 20 + i), seeded((2, 4, 3, 64, 64), 30 + i), torch.tensor([i % 2, 1]),
                 torch.ones(2, 4), torch.ones(2, 4))
        loss, logits, probs = tr.micro_step(i, 8, batch)
        assert torch.isfinite(loss) and logits.shape == (2, 2) and probs.shape == (2,)
        if i < 3:
            assert all(torch.equal(p, b) for p, b in zip(m.parameters(), before))
    torch.cuda.synchronize()
    assert tr.scaler.get_scale() == 2.0 ** 8, f"the scaler skipped the step (scale now {tr.scaler.get_scale()})"
    assert not all(torch.equal(p, b) for p, b in zip(m.parameters(), before))
    assert tr.optimizer_steps == 1 and int(tr.ema_model.n_averaged) == 1 and tr.optimizer.param_groups[0]["lr"] != lr0
    for pa, pm in zip(tr.ema_model.module.parameters(), m.parameters()):
        assert torch.equal(pa, pm)
    s = tr.eval_scores((seeded((2, 3, 3, 64, 64), 40), seeded((2, 4, 3, 64, 64), 41), torch.tensor([0, 1])))
    assert s.shape == (2,) and bool(((s >= 0) & (s <= 1)).all())
