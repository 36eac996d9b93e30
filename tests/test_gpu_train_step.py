"""GPU: the heads / losses on their HIP kernels, and the reference's active training steps.

* ArcFaceHead / CBFocalLoss / cross_entropy (csrc/heads.hip) against the reference classes'
  goldens (heads.npz): logits, loss and input / weight gradients, fp32 (rel 1e-5; acos / cos
  on the device vs glibc).
* The train_visual.py:563-577 step (arcface_step.npz, captured from the reference on CPU):
  extract_features(x, seq_lengths) -> model.lstm(f)[0][:, -1] -> ArcFaceHead(128, 2, s=30,
  m=0.5) -> CrossEntropyLoss -> backward -> clip_grad_norm_(1.0) -> Adam(lr 1e-5, wd 1e-4)
  over model + head parameters, at the reference's frame sizes 224^2 and 256^2, frozen and
  unfrozen backbone, fp32 (the contract of test_gpu_model.py).
* The same step as the script runs it on a GPU: under autocast("cuda") with a GradScaler
  (the backbone then computes in bf16, the head and losses in fp32), against the oracle's
  fp32 emulation of exactly that sequence (loss x scale -> backward -> clip_grad_norm_ on
  the scaled gradients, as the script does -> unscale -> Adam), bf16 tolerances.
"""
import numpy as np
import pytest
import torch
import torch.nn as nn

pytestmark = pytest.mark.gpu


def seeded_uniform(shape, seed):
    return torch.rand(shape, generator=torch.Generator().manual_seed(seed), dtype=torch.float32)


def relerr(a, b):
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    return float(np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-30))


@pytest.mark.parametrize("tag", ["v", "a"])
def test_heads_vs_reference(gpu, golden, tag):
    from xcp.heads import ArcFaceHead, CBFocalLoss, cross_entropy
    g = golden("heads.npz")
    m_ = 0.5 if tag == "v" else 0.30
    head = ArcFaceHead(128, 2, s=30.0, m=m_).to(gpu)
    with torch.no_grad():
        head.weight.copy_(torch.tensor(g[f"{tag}/weight"]))
    f = torch.tensor(g[f"{tag}/features"]).to(gpu).requires_grad_(True)
    lab = torch.tensor(g[f"{tag}/labels"]).long().to(gpu)
    np.testing.assert_allclose(head(f).detach().cpu().numpy(), g[f"{tag}/logits_nolabel"], rtol=1e-5, atol=1e-5)
    logits = head(f, lab)
    np.testing.assert_allclose(logits.detach().cpu().numpy(), g[f"{tag}/logits"], rtol=1e-5, atol=1e-5)
    if tag == "v":
        loss = cross_entropy(logits, lab)
        np.testing.assert_allclose(loss.item(), nn.CrossEntropyLoss()(logits.detach(), lab).item(), rtol=1e-6)
    else:
        loss = CBFocalLoss([300, 1700], beta=0.9999, gamma=2.0).to(gpu)(logits, lab)
    loss.backward()
    torch.cuda.synchronize()
    np.testing.assert_allclose(loss.item(), g[f"{tag}/loss"], rtol=1e-5)
    assert relerr(f.grad.cpu(), g[f"{tag}/dfeatures"]) < 1e-5
    assert relerr(head.weight.grad.cpu(), g[f"{tag}/dweight"]) < 1e-5
    # row 0 sits exactly on its class centre (cos = 1): the clamp zeroes its target-logit gradient
    assert np.isfinite(f.grad.cpu().numpy()).all()


def _visual_step(gpu, S, mode, T, B, autocast=False):
    import xcp
    from xcp.heads import ArcFaceHead
    from xcp.optim import FusedAdamClip
    from Models.XceptionLSTMV import XceptionLSTMV
    torch.manual_seed(0)
    m = XceptionLSTMV(128, pretrained=False)
    torch.manual_seed(1)
    head = ArcFaceHead(128, 2, s=30.0, m=0.5)
    for p in m.feature_extractor.parameters():
        p.requires_grad = mode == "unfrozen"
    m, head = m.to(gpu).train(), head.to(gpu).train()
    x = seeded_uniform((B, T, 3, S, S), 6000 + S).to(gpu)
    lab = torch.tensor([0, 1], device=gpu)[:B]
    seq_lengths = torch.full((B,), T, device=gpu)
    params = list(m.parameters()) + list(head.parameters())
    opt = FusedAdamClip(params, lr=1e-5, weight_decay=1e-4)
    criterion = nn.CrossEntropyLoss()
    out = {}
    opt.zero_grad()
    if autocast:
        scaler = torch.amp.GradScaler()
        with torch.autocast("cuda"):
            feats = m.extract_features(x, seq_lengths)
            emb = m.lstm(feats)[0][:, -1, :]
            logits = head(emb, lab)
            loss = criterion(logits, lab)
        scaler.scale(loss).backward()
        out["total"] = torch.nn.utils.clip_grad_norm_(params, 1.0).item()
        scaler.step(opt)
        scaler.update()
        out["scale"] = scaler.get_scale()
    else:
        with xcp.precision("fp32"):
            feats = m.extract_features(x, seq_lengths)
            emb = m.lstm(feats)[0][:, -1, :]
            logits = head(emb, lab)
            loss = criterion(logits, lab)
            loss.backward()
        out["grads"] = {n: p.grad.detach().clone() for n, p in m.named_parameters() if p.grad is not None}
        out["head_grad"] = head.weight.grad.detach().clone()
        out["total"] = torch.nn.utils.clip_grad_norm_(params, 1.0).item()
        opt.step()
    torch.cuda.synchronize()
    out.update(m=m, head=head, logits=logits.detach().float(), emb=emb.detach().float(), loss=loss.item())
    return out


@pytest.mark.parametrize("S,mode", [(224, "unfrozen"), (224, "frozen"), (256, "unfrozen")])
def test_train_visual_arcface_step_fp32(gpu, golden, S, mode):
    g = golden("arcface_step.npz")
    B, T = int(g["B"]), int(g["T"])
    tag = f"s{S}_{mode}"
    r = _visual_step(gpu, S, mode, T, B)
    np.testing.assert_allclose(r["emb"].cpu().numpy(), g[f"{tag}/emb"], rtol=1e-4, atol=1e-6)
    np.testing.assert_allclose(r["logits"].cpu().numpy(), g[f"{tag}/logits"], rtol=1e-4, atol=1e-4)
    np.testing.assert_allclose(r["loss"], g[f"{tag}/loss"], rtol=1e-5)
    for n, gr in r["grads"].items():
        e = abs(gr.double().norm().item() - g[f"{tag}/gradnorm/{n}"]) / g[f"{tag}/gradnorm/{n}"]
        assert e < (5e-3 if gr.dim() == 1 and "feature_extractor" in n else 1e-3), (n, e)
    assert {n for n in r["grads"]} == {k.split("/", 2)[2] for k in g if k.startswith(f"{tag}/gradnorm/")} - {
        "head.weight"}
    e = abs(r["head_grad"].double().norm().item() - g[f"{tag}/gradnorm/head.weight"]) / g[f"{tag}/gradnorm/head.weight"]
    assert e < 1e-3, e
    np.testing.assert_allclose(r["total"], g[f"{tag}/total_gradnorm"], rtol=1e-3)
    for n, p in r["m"].named_parameters():
        got, want = p.detach().double().sum().item(), float(g[f"{tag}/after_step/{n}/sum"])
        tol = 2 * 1e-5 * max(5e-3 * p.numel(), 2) + 1e-6 * abs(want) + 1e-7   # 0.5 % sign flips of Adam's step
        assert abs(got - want) <= tol, (n, got, want, tol)
    np.testing.assert_allclose(r["head"].weight.detach().cpu().numpy(), g[f"{tag}/after_step/head.weight"], rtol=1e-5,
                               atol=1e-7)


def test_train_visual_step_autocast_gradscaler(gpu):
    """The script's own GPU sequence (autocast fp16 -> xcp backbone in bf16, GradScaler, clip of
    the SCALED gradients to 1.0, scaler.step(FusedAdamClip)) against the oracle emulating it in
    fp32 on the CPU.  The scale survives (no inf); the loss agrees to 2e-2; the parameters
    after the step agree as test_gpu_model's bf16 after-step contract (head: 10 % sign flips of
    Adam's first update allowed, backbone 20 %)."""
    from oracle import xception_oracle as O
    B, T, S = 2, 3, 224
    r = _visual_step(gpu, S, "unfrozen", T, B, autocast=True)
    assert r["scale"] == 65536.0
    # oracle: the same step in fp32 on the CPU
    from Models.XceptionLSTMV import XceptionLSTMV
    from xcp.heads import ArcFaceHead
    torch.manual_seed(0)
    sd = XceptionLSTMV(128, pretrained=False).state_dict()
    torch.manual_seed(1)
    w = ArcFaceHead(128, 2).weight.detach().clone()
    params = {k: v.clone().requires_grad_(v.is_floating_point() and "running" not in k) for k, v in sd.items()}
    w.requires_grad_(True)
    x = seeded_uniform((B, T, 3, S, S), 6000 + S)
    lab = torch.tensor([0, 1])
    feats = O.backbone_forward(x.reshape(B * T, 3, S, S), params, True, {}, prefix="feature_extractor.").view(B, T, -1)
    out, _, _ = O.lstm_forward(feats, params["lstm.weight_ih_l0"], params["lstm.weight_hh_l0"],
                               params["lstm.bias_ih_l0"], params["lstm.bias_hh_l0"])
    logits = O.arcface_logits(out[:, -1, :], w, lab, 30.0, 0.5)
    loss = nn.CrossEntropyLoss()(logits, lab)
    (loss * 65536.0).backward()
    train = {k: v for k, v in params.items() if v.requires_grad and v.grad is not None}   # (fc_layers / fc_out
    train["head.weight"] = w                                                              # are unused here)
    grads = {k: v.grad for k, v in train.items()}
    total = O.clip_grad_norm(list(grads.values()), 1.0)
    for gr in grads.values():
        gr.div_(65536.0)
    O.adam_step(train, grads, {}, 1e-5, weight_decay=1e-4)
    np.testing.assert_allclose(r["loss"], loss.item(), rtol=2e-2)
    np.testing.assert_allclose(r["total"], total.item(), rtol=5e-2)
    bad = []
    for n, p in list(r["m"].named_parameters()) + [("head.weight", r["head"].weight)]:
        if n not in train:
            continue
        got, want = p.detach().double().sum().item(), train[n].detach().double().sum().item()
        frac = 0.2 if n.startswith("feature_extractor.") else 0.1
        tol = 2 * 1e-5 * max(frac * p.numel(), 2) + 1e-6 * abs(want) + 1e-7
        if abs(got - want) > tol:
            bad.append((n, got, want, tol))
    assert not bad, bad[:5]


def test_second_step_forward_uses_updated_weights(gpu):
    """Two FusedAdamClip training steps (fp32): the second forward runs on the weights the first
    step wrote (the engine repacks its kernel-layout copies when the optimiser bumps the parameter
    versions) -- its output equals that of a fresh model loaded with the post-step state_dict, and
    differs from the first forward's."""
    import xcp
    from xcp.optim import FusedAdamClip
    from Models.Xception import xception
    torch.manual_seed(0)
    m = xception(num_classes=1).to(gpu).train()
    opt = FusedAdamClip(m.parameters(), lr=1e-2, max_norm=1.0)
    x = seeded_uniform((2, 3, 96, 96), 77).to(gpu)
    outs = []
    with xcp.precision("fp32"):
        for _ in range(2):
            out = m(x)
            outs.append(out.detach().clone())
            out.sum().backward()
            opt.step()
            opt.zero_grad()
        sd = {k: v.clone() for k, v in m.state_dict().items()}
        m.eval()
        got = m(x).detach()
        fresh = xception(num_classes=1).to(gpu)
        fresh.load_state_dict(sd)
        fresh.eval()
        want = fresh(x).detach()
    torch.cuda.synchronize()
    assert not torch.equal(outs[0], outs[1])
    torch.testing.assert_close(got, want, rtol=0, atol=0)


def test_fused_adam_capturable_matches_eager(gpu):
    """FusedAdamClip(capturable=True) -- device step counts, bias corrections formed on the device --
    captured in a HIP graph and replayed gives bit for bit the eager optimiser's parameters, moments
    and step count (clip on)."""
    from xcp.optim import FusedAdamClip
    g = torch.Generator(device=gpu).manual_seed(5)
    shapes = [(700, 33), (5,), (64, 3, 3, 3), (40000,)]
    init = [torch.randn(s, device=gpu, generator=g) for s in shapes]
    grads = [torch.randn(s, device=gpu, generator=g) for s in shapes]
    pa = [t.clone().requires_grad_(True) for t in init]
    pb = [t.clone().requires_grad_(True) for t in init]
    for p, q, gr in zip(pa, pb, grads):
        p.grad, q.grad = gr.clone(), gr.clone()
    oa = FusedAdamClip(pa, lr=1e-2, weight_decay=1e-4, max_norm=1.0)
    ob = FusedAdamClip(pb, lr=1e-2, weight_decay=1e-4, max_norm=1.0, capturable=True)
    for _ in range(4):
        oa.step()
    ob.step()   # eager (creates the state and the tables), then one captured step replayed three times
    s = torch.cuda.Stream(gpu)
    s.wait_stream(torch.cuda.current_stream())
    torch.cuda.synchronize()
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph):
        ob.step()
    for _ in range(3):
        graph.replay()
    torch.cuda.synchronize()
    for p, q in zip(pa, pb):
        assert torch.equal(p, q)
        assert torch.equal(oa.state[p]["exp_avg"], ob.state[q]["exp_avg"])
        assert torch.equal(oa.state[p]["exp_avg_sq"], ob.state[q]["exp_avg_sq"])
        assert float(ob.state[q]["step"]) == 4.0


def test_graph_captured_train_step_matches_eager(gpu):
    """The bench's graph mode: a whole xception(num_classes=1) train step (bf16 engine forward and
    backward with the side-stream weight gradients, BCE, clip + Adam with device step counts) captured
    as one HIP graph and replayed gives bit for bit the parameters and BatchNorm buffers of the same
    steps run eagerly."""
    import xcp
    from torch.autograd.graph import increment_version
    from xcp.optim import FusedAdamClip
    from Models.Xception import xception
    x = seeded_uniform((4, 3, 96, 96), 31).to(gpu)
    y = torch.tensor([[0.0], [1.0], [1.0], [0.0]], device=gpu)
    models = []
    for capt in (False, True):
        torch.manual_seed(0)
        m = xception(num_classes=1).to(gpu).train()
        opt = FusedAdamClip(m.parameters(), lr=1e-3, weight_decay=1e-4, max_norm=1.0, capturable=capt)

        def step():
            opt.zero_grad(set_to_none=False)
            nn.BCEWithLogitsLoss()(m(x), y).backward()
            opt.step()

        with xcp.precision("bf16"):
            if not capt:
                for _ in range(4):
                    step()
            else:
                step()   # eager warm-up: persistent buffers, packs, optimiser tables
                torch.cuda.synchronize()
                graph = torch.cuda.CUDAGraph()
                with torch.cuda.graph(graph):
                    step()
                for _ in range(3):
                    graph.replay()
                    increment_version(list(m.parameters()))
        torch.cuda.synchronize()
        models.append(m)
    sa, sb = models[0].state_dict(), models[1].state_dict()
    for k in sa:
        assert torch.equal(sa[k], sb[k]), k


@pytest.mark.parametrize("flag", ["WGRAD_DEFER", "WGRAD_FIRST", "SKIP_WGRAD_LATE"])
def test_wgrad_schedule_switches_bitwise(gpu, monkeypatch, flag):
    """The engine's side-stream schedule switches (a unit's weight gradient launched before its input gradient,
    after the next unit's, the skip conv's after the block) only reorder independent launches: every gradient
    of a bf16 xception backward is bit for bit the default schedule's."""
    import xcp
    from xcp import engine
    from Models.Xception import xception
    x = seeded_uniform((4, 3, 96, 96), 37).to(gpu)
    grads = []
    for on in (False, True):
        monkeypatch.setattr(engine, flag, on)
        torch.manual_seed(0)
        m = xception(num_classes=1).to(gpu).train()
        with xcp.precision("bf16"):
            m(x).float().square().sum().backward()
        torch.cuda.synchronize()
        grads.append({n: p.grad.clone() for n, p in m.named_parameters()})
    for n in grads[0]:
        assert torch.equal(grads[0][n], grads[1][n]), n


@pytest.mark.parametrize("B", [2, 16])
def test_graph_captured_lstma_step_matches_eager(gpu, B):
    """The C4 line's default execution (bench.py --model lstma: one HIP graph per step): an XceptionLSTMA(512)
    train step with the frozen backbone (bf16 engine forward, the H = 512 LSTM on its persistent forward and --
    B 2 -- the clip-grouped persistent backward or -- B 16 -- the per-step backward, BCE, clip + Adam with device
    step counts) captured and replayed gives bit for bit the parameters of the same steps run eagerly, and no
    persistent launch reports a poll timeout."""
    import xcp
    from torch.autograd.graph import increment_version
    from xcp import ops
    from xcp.optim import FusedAdamClip
    from Models.XceptionLSTMA import XceptionLSTMA
    x = seeded_uniform((B, 12, 3, 13), 41).to(gpu) * 2.0 - 1.0
    y = (torch.arange(B, device=gpu) % 2).float().view(B, 1)
    models = []
    for capt in (False, True):
        torch.manual_seed(0)
        m = XceptionLSTMA(512, pretrained=False).to(gpu).train()
        for p in m.feature_extractor.parameters():
            p.requires_grad = False
        params = [p for p in m.parameters() if p.requires_grad]
        opt = FusedAdamClip(params, lr=1e-4, weight_decay=0.0, max_norm=1.0, capturable=capt)

        def step():
            opt.zero_grad(set_to_none=False)
            nn.BCELoss()(m(m.extract_features(x, gpu)), y).backward()
            opt.step()

        with xcp.precision("bf16"):
            if not capt:
                for _ in range(4):
                    step()
            else:
                step()
                torch.cuda.synchronize()
                graph = torch.cuda.CUDAGraph()
                with torch.cuda.graph(graph):
                    step()
                for _ in range(3):
                    graph.replay()
                    increment_version(params)
        torch.cuda.synchronize()
        models.append(m)
    assert ops.lstm_sync_error() == 0
    sa, sb = models[0].state_dict(), models[1].state_dict()
    for k in sa:
        assert torch.equal(sa[k], sb[k]), k


def test_fused_adam_capturable_late_parameter_vs_torch(gpu):
    """A parameter whose first gradient arrives at step 3 (the reference's unfreeze after epoch 3,
    train_visual.py:547-556) and one that skips a step keep their own step counts under
    capturable=True, as in torch.optim.Adam(capturable=True) (advisor round 4)."""
    from xcp.optim import FusedAdamClip
    g = torch.Generator(device=gpu).manual_seed(9)
    shapes = [(300, 7), (64,), (32, 3, 3, 3)]
    init = [torch.randn(s, device=gpu, generator=g) for s in shapes]
    pa = [t.clone().requires_grad_(True) for t in init]
    pb = [t.clone().requires_grad_(True) for t in init]
    ref = torch.optim.Adam(pa, lr=1e-2, weight_decay=1e-4, capturable=True)
    opt = FusedAdamClip(pb, lr=1e-2, weight_decay=1e-4, capturable=True)
    for k in range(6):
        for i, (p, q) in enumerate(zip(pa, pb)):
            skip = (i == 1 and k < 2) or (i == 2 and k == 3)
            gr = None if skip else torch.randn(shapes[i], device=gpu, generator=g)
            p.grad = None if gr is None else gr.clone()
            q.grad = None if gr is None else gr.clone()
        ref.step()
        opt.step()
    torch.cuda.synchronize()
    for p, q in zip(pa, pb):
        torch.testing.assert_close(q, p, rtol=1e-5, atol=1e-6)
        assert float(opt.state[q]["step"]) == float(ref.state[p]["step"])
