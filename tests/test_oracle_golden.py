"""Pin the CPU oracle (oracle/xception_oracle.py) against golden vectors captured from
the reference itself (tools/capture_goldens.py, torch 2.10.0 CPU).  CPU only."""
import numpy as np
import pytest
import torch
import torch.nn as nn

from Models.Xception import Block, SeparableConv2d, xception
from Models.XceptionLSTMA import XceptionLSTMA
from Models.XceptionLSTMV import XceptionLSTMV
from oracle import xception_oracle as O


def seeded_uniform(shape, seed):
    return torch.rand(shape, generator=torch.Generator().manual_seed(seed), dtype=torch.float32)


def seeded_normal(shape, seed):
    return torch.randn(shape, generator=torch.Generator().manual_seed(seed), dtype=torch.float32)


def check_fp(g, prefix, t, rtol=1e-5, atol=1e-5):
    a = t.detach().double().reshape(-1).numpy()
    assert tuple(g[f"{prefix}/shape"]) == tuple(t.shape)
    np.testing.assert_allclose(a[g[f"{prefix}/idx"]], g[f"{prefix}/val"], rtol=rtol, atol=atol)
    np.testing.assert_allclose(a.sum(), g[f"{prefix}/sum"], rtol=1e-4, atol=1e-3)
    np.testing.assert_allclose((a * a).sum(), g[f"{prefix}/sumsq"], rtol=1e-5)


def backbone_sd(seed=0):
    torch.manual_seed(seed)
    m = xception(num_classes=1000)
    return {k: v.clone() for k, v in m.state_dict().items() if not k.startswith("fc.")}


def test_backbone64_train_forward_backward(golden):
    g = golden("backbone64.npz")
    sd = backbone_sd()
    params = {k: v.clone().requires_grad_(("running" not in k and "num_batches" not in k)) for k, v in sd.items()}
    x = seeded_uniform((4, 3, 64, 64), 1234)
    stats = {}
    f = O.backbone_forward(x, params, True, stats)
    np.testing.assert_allclose(f.detach().numpy(), g["features"], rtol=1e-5, atol=1e-6)
    r = seeded_normal(f.shape, 99)
    (f * r).sum().backward()
    for k, p in params.items():
        key = f"gradnorm/{k}"
        if key in g:
            np.testing.assert_allclose(p.grad.double().norm().item(), g[key], rtol=1e-4, err_msg=k)
    np.testing.assert_allclose(params["conv1.weight"].grad.numpy(), g["grad/conv1.weight"], rtol=1e-4, atol=1e-6)
    np.testing.assert_allclose(params["bn4.weight"].grad.numpy(), g["grad/bn4.weight"], rtol=1e-4, atol=1e-6)
    for k, v in stats.items():
        if "running" in k:
            np.testing.assert_allclose(v.double().sum().item(), g[f"buf/{k}/sum"], rtol=1e-5, atol=1e-6, err_msg=k)
    sd2 = dict(sd)
    sd2.update({k: v for k, v in stats.items() if v is not None})
    with torch.no_grad():
        fe = O.backbone_forward(x, sd2, False)
    np.testing.assert_allclose(fe.numpy(), g["features_eval"], rtol=1e-4, atol=1e-5)


@pytest.mark.parametrize("H,T", [(128, 16), (512, 12)])
def test_lstm(golden, H, T):
    g = golden("lstm.npz")
    torch.manual_seed(0)
    lstm = nn.LSTM(2048, H, 1, batch_first=True)
    w = {n: p.detach().clone().requires_grad_(True) for n, p in lstm.named_parameters()}
    x = seeded_normal((2, T, 2048), 555).requires_grad_(True)
    o, h, c = O.lstm_forward(x, w["weight_ih_l0"], w["weight_hh_l0"], w["bias_ih_l0"], w["bias_hh_l0"])
    p = f"H{H}"
    np.testing.assert_allclose(o.detach().numpy(), g[f"{p}/out"], rtol=1e-5, atol=1e-6)
    np.testing.assert_allclose(h.detach().numpy(), g[f"{p}/h_n"], rtol=1e-5, atol=1e-6)
    np.testing.assert_allclose(c.detach().numpy(), g[f"{p}/c_n"], rtol=1e-5, atol=1e-6)
    r = seeded_normal(o.shape, 556)
    rh = seeded_normal(h.shape, 557)
    ((o * r).sum() + (c * rh).sum()).backward()
    np.testing.assert_allclose(x.grad.numpy(), g[f"{p}/dx"], rtol=1e-4, atol=1e-6)
    for n, t in w.items():
        ref = g[f"{p}/grad/{n}"]
        if ref.ndim == 0:
            np.testing.assert_allclose(t.grad.double().norm().item(), ref, rtol=1e-5)
        else:
            np.testing.assert_allclose(t.grad.numpy(), ref, rtol=1e-4, atol=1e-6)


def test_blocks(golden):
    g = golden("blocks.npz")
    for i, name in enumerate(["block1", "block4", "block12"]):
        cin, cout, reps, s, swr, gf, hw = [int(v) for v in g[f"{name}/cfg"]]
        torch.manual_seed(10 + i)
        blk = Block(cin, cout, reps, s, start_with_relu=bool(swr), grow_first=bool(gf))
        for mm in blk.modules():
            if isinstance(mm, nn.Conv2d):
                n = mm.kernel_size[0] * mm.kernel_size[1] * mm.out_channels
                mm.weight.data.normal_(0, (2.0 / n) ** 0.5)
        params = {k: v.clone().requires_grad_("running" not in k and "num_batches" not in k)
                  for k, v in blk.state_dict().items()}
        x = seeded_normal((2, cin, hw, hw), 100 + i).requires_grad_(True)
        stats = {}
        y = O.block_forward(x, {f"b.{k}": v for k, v in params.items()}, "b", (cin, cout, reps, s, bool(swr), bool(gf)),
                            True, stats)
        r = seeded_normal(y.shape, 200 + i)
        (y * r).sum().backward()
        check_fp(g, f"{name}/out", y)
        check_fp(g, f"{name}/dx", x.grad, rtol=1e-4, atol=1e-5)
        for k, p in params.items():
            key = f"{name}/gradnorm/{k}"
            if key in g:
                np.testing.assert_allclose(p.grad.double().norm().item(), g[key], rtol=1e-4, err_msg=k)


def test_sepconv(golden):
    g = golden("sepconv.npz")
    for key in sorted({k.split("/")[0] for k in g if k.startswith("s")}):
        cin, cout, hw, sw, sx, sr = [int(v) for v in g[f"{key}/cfg"]]
        torch.manual_seed(sw)
        sc = SeparableConv2d(cin, cout, 3, 1, 1)
        sd = {f"s.{k}": v.clone().requires_grad_(True) for k, v in sc.state_dict().items()}
        x = seeded_normal((2, cin, hw, hw), sx).requires_grad_(True)
        y = O.sepconv(x, sd, "s")
        (y * seeded_normal(y.shape, sr)).sum().backward()
        check_fp(g, f"{key}/y", y, rtol=1e-4, atol=1e-5)
        check_fp(g, f"{key}/dx", x.grad, rtol=1e-4, atol=1e-5)
        np.testing.assert_allclose(sd["s.conv1.weight"].grad.numpy(), g[f"{key}/dw_grad"], rtol=1e-4, atol=1e-5)
        np.testing.assert_allclose(sd["s.pointwise.weight"].grad.double().norm().item(), g[f"{key}/pw_gradnorm"],
                                   rtol=1e-5)


def _clip_sd(model_cls, hidden):
    torch.manual_seed(0)
    m = model_cls(hidden, pretrained=False)
    return m.state_dict()


@pytest.mark.parametrize("mode", ["frozen", "unfrozen"])
def test_lstmv_clip_step(golden, mode):
    g = golden("lstmv_b2t4.npz")
    B, T, S = int(g["B"]), int(g["T"]), int(g["S"])
    x = seeded_uniform((B, T, 3, S, S), 1234)
    y = torch.tensor([[0.0], [1.0]])[:B]
    r = O.clip_step(_clip_sd(XceptionLSTMV, 128), x, y, unfrozen=(mode == "unfrozen"))
    np.testing.assert_allclose(r["features"].numpy(), g[f"{mode}/features"], rtol=1e-4, atol=1e-5)
    np.testing.assert_allclose(r["logits"].numpy(), g[f"{mode}/logits"], rtol=1e-5, atol=1e-6)
    np.testing.assert_allclose(r["prob"].numpy(), g[f"{mode}/prob"], rtol=1e-6, atol=1e-7)
    np.testing.assert_allclose(r["loss"].item(), g[f"{mode}/loss"], rtol=1e-6)
    tot = 0.0
    for k, gr in r["grads"].items():
        key = f"{mode}/gradnorm/{k}"
        assert key in g, k
        np.testing.assert_allclose(gr.double().norm().item(), g[key], rtol=1e-3, err_msg=k)
        tot += (gr.double() ** 2).sum().item()
    np.testing.assert_allclose(tot ** 0.5, g[f"{mode}/total_gradnorm"], rtol=1e-4)


def test_audio_clip(golden):
    g = golden("audio_b2t6.npz")
    B, T = int(g["B"]), int(g["T"])
    x = seeded_normal((B, T, 3, 13), 777)
    frames = O.audio_frames(x)
    check_fp(g, "frames_fp", frames, rtol=1e-6, atol=1e-6)
    y = torch.tensor([[1.0], [0.0]])[:B]
    r = O.clip_step(_clip_sd(XceptionLSTMA, 512), x, y, unfrozen=False, audio=True)
    np.testing.assert_allclose(r["features"].numpy(), g["features"], rtol=1e-4, atol=1e-5)
    np.testing.assert_allclose(r["logits"].numpy(), g["logits"], rtol=1e-5, atol=1e-6)
    np.testing.assert_allclose(r["loss"].item(), g["loss"], rtol=1e-6)
    for k, gr in r["grads"].items():
        np.testing.assert_allclose(gr.double().norm().item(), g[f"gradnorm/{k}"], rtol=1e-3, err_msg=k)


def test_oracle_optimizer_step_vs_reference(golden):
    """oracle.clip_grad_norm + oracle.adam_step against the reference's own step at the bench
    kernel-set size (lstmv_b4t16.npz: clip_grad_norm_(1.0) + Adam(lr 1e-5, wd 1e-4),
    train_visual.py:533, :575-577), parameter sums after the step."""
    g = golden("lstmv_b4t16.npz")
    B, T, S = int(g["B"]), int(g["T"]), int(g["S"])
    x = seeded_uniform((B, T, 3, S, S), 4242)
    y = torch.tensor([[0.0], [1.0], [1.0], [0.0]])[:B]
    torch.manual_seed(0)
    sd = XceptionLSTMV(128, pretrained=False).state_dict()
    r = O.clip_step(sd, x, y, unfrozen=True, optim=dict(lr=1e-5, weight_decay=1e-4, max_norm=1.0))
    np.testing.assert_allclose(r["loss"].item(), g["loss"], rtol=1e-6)
    for k, p in r["params"].items():
        key = f"after_step/{k}/sum"
        if key in g:
            a = p.detach().double()
            np.testing.assert_allclose(a.sum().item(), g[key], rtol=1e-6, atol=2e-5 * 1e-3 * a.numel() + 1e-6,
                                       err_msg=k)
            np.testing.assert_allclose((a * a).sum().item(), g[f"after_step/{k}/sumsq"], rtol=1e-5, err_msg=k)


def test_frame_step_c1(golden):
    """Config C1 (xception(num_classes=1), B = 4 frames of 299^2, BCEWithLogits + Adam): the
    oracle's frame_step against the reference's own step (xception_c1_b4.npz)."""
    g = golden("xception_c1_b4.npz")
    B, S = int(g["B"]), int(g["S"])
    torch.manual_seed(0)
    sd = {k: v.clone() for k, v in xception(num_classes=1).state_dict().items()}
    x = seeded_uniform((B, 3, S, S), int(g["seed_x"]))
    y = (torch.arange(B) % 3 == 0).float().view(B, 1)
    r = O.frame_step(sd, x, y, optim=dict(lr=float(g["lr"]), weight_decay=float(g["weight_decay"])))
    np.testing.assert_allclose(r["logits"].numpy(), g["logits"], rtol=0, atol=1e-5)
    np.testing.assert_allclose(r["loss"].item(), g["loss"], rtol=1e-6)
    for n, gr in r["grads"].items():
        np.testing.assert_allclose(gr.double().norm().item(), g[f"gradnorm/{n}"], rtol=1e-4, err_msg=n)
    for n, p in r["params"].items():
        if f"after_step/{n}/sum" in g:
            np.testing.assert_allclose(p.detach().double().sum().item(), g[f"after_step/{n}/sum"], rtol=1e-6,
                                       atol=1e-6, err_msg=n)


def test_oracle_lstm_t120(golden):
    """oracle.lstm_forward over XceptionLSTMA's own recurrence (H = 512, T = 120,
    audio_dataloader.py:20,39) against the reference nn.LSTM (lstm_t120.npz), including the
    per-time-step output norms and the backward through all 120 steps."""
    g = golden("lstm_t120.npz")
    B, T, H = int(g["B"]), int(g["T"]), int(g["H"])
    torch.manual_seed(0)
    ref = nn.LSTM(2048, H, 1, batch_first=True)
    cp = {n: p.detach().clone().requires_grad_(True) for n, p in ref.named_parameters()}
    x = seeded_normal((B, T, 2048), 555).requires_grad_(True)
    o, h, c = O.lstm_forward(x, cp["weight_ih_l0"], cp["weight_hh_l0"], cp["bias_ih_l0"], cp["bias_hh_l0"])
    check_fp(g, "out", o, rtol=1e-5, atol=1e-6)
    np.testing.assert_allclose(o.detach().double().norm(dim=2).numpy(), g["out_step_norm"], rtol=1e-5)
    np.testing.assert_allclose(h.detach().numpy(), g["h_n"], rtol=1e-5, atol=1e-6)
    np.testing.assert_allclose(c.detach().numpy(), g["c_n"], rtol=1e-5, atol=1e-6)
    ((o * seeded_normal(o.shape, 556)).sum() + (c * seeded_normal(c.shape, 557)).sum()).backward()
    check_fp(g, "dx", x.grad, rtol=1e-4, atol=1e-6)
    for n, p in cp.items():
        np.testing.assert_allclose(p.grad.double().norm().item(), g[f"gradnorm/{n}"], rtol=1e-5, err_msg=n)


def test_audio_clip_t120(golden):
    """oracle.clip_step on the XceptionLSTMA step at T = 120 (audio_b2t120.npz, frozen backbone as
    shipped): 240 frames of 64^2, then H = 512 over 120 steps."""
    g = golden("audio_b2t120.npz")
    B, T = int(g["B"]), int(g["T"])
    x = seeded_normal((B, T, 3, 13), 778)
    y = torch.tensor([[1.0], [0.0]])[:B]
    r = O.clip_step(_clip_sd(XceptionLSTMA, 512), x, y, unfrozen=False, audio=True)
    check_fp(g, "frozen/features", r["features"], rtol=1e-4, atol=1e-5)
    np.testing.assert_allclose(r["logits"].numpy(), g["frozen/logits"], rtol=1e-5, atol=1e-6)
    np.testing.assert_allclose(r["loss"].item(), g["frozen/loss"], rtol=1e-6)
    for k, gr in r["grads"].items():
        np.testing.assert_allclose(gr.double().norm().item(), g[f"frozen/gradnorm/{k}"], rtol=1e-3, err_msg=k)
