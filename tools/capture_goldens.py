"""Capture golden vectors from the reference implementation (run in the build container ONLY).

The reference (Tonmoy1321/Multimodal-DeepFake-Detection, mounted read-only at
/root/reference) is imported offline exactly as SURVEY.md §8(c) describes:

* a synthetic package ``refpkg`` whose ``__path__`` is ``/root/reference`` so the
  package-relative ``from .Xception import xception`` in XceptionLSTMV.py:5 /
  XceptionLSTMA.py:3 resolves;
* ``Xception.model_zoo.load_url`` is stubbed to raise (Xception.py:212 would fetch
  pretrained weights over the network), and ``xception`` is rebound inside the
  V/A modules to ``pretrained=False`` (XceptionLSTMV.py:12, XceptionLSTMA.py:8),
  so goldens use the seeded init of Xception.py:154-160;
* ``sys.dont_write_bytecode`` because the reference directory is read-only.

Only the resulting ``tests/golden/*.npz`` fixtures (inputs are regenerated from
the recorded seeds; outputs, fingerprints and small full tensors are stored) are
committed.  Neither the reference nor this script is needed on the GPU box.

Usage:  python tools/capture_goldens.py  [--out tests/golden]
"""
import argparse
import importlib.util
import os
import sys
import types

import numpy as np
import torch
import torch.nn as nn
import torch.nn.functional as F

REF = "/root/reference"
sys.dont_write_bytecode = True
torch.set_num_threads(max(1, os.cpu_count() or 1))


def load_reference():
    pkg = types.ModuleType("refpkg")
    pkg.__path__ = [REF]
    sys.modules["refpkg"] = pkg

    def load(name):
        spec = importlib.util.spec_from_file_location(f"refpkg.{name}", os.path.join(REF, f"{name}.py"))
        mod = importlib.util.module_from_spec(spec)
        sys.modules[f"refpkg.{name}"] = mod
        spec.loader.exec_module(mod)
        return mod

    X = load("Xception")

    def _no_fetch(*a, **k):
        raise RuntimeError("network fetch of pretrained weights is disabled")

    X.model_zoo.load_url = _no_fetch
    V = load("XceptionLSTMV")
    A = load("XceptionLSTMA")
    offline = lambda pretrained=False, **kw: X.xception(pretrained=False, **kw)  # noqa: E731
    V.xception = offline
    A.xception = offline
    return X, V, A


# ----------------------------------------------------------------------------- helpers
def fp(t, n_samples=4096, seed=7):
    """Fingerprint of a tensor: sum, sum of squares (fp64), and n seeded samples."""
    a = t.detach().double().cpu().numpy().reshape(-1)
    rs = np.random.RandomState(seed)
    idx = rs.choice(a.size, size=min(n_samples, a.size), replace=False) if a.size else np.zeros(0, np.int64)
    idx = np.sort(idx)
    return {"sum": a.sum(), "sumsq": (a * a).sum(), "idx": idx.astype(np.int64), "val": a[idx].astype(np.float64),
            "shape": np.array(t.shape, dtype=np.int64)}


def put_fp(out, prefix, t, **kw):
    for k, v in fp(t, **kw).items():
        out[f"{prefix}/{k}"] = v


def state_fp(out, prefix, module):
    for name, t in module.state_dict().items():
        if t.dtype in (torch.float32, torch.float64):
            a = t.detach().double().reshape(-1)
            out[f"{prefix}/{name}/sum"] = a.sum().item()
            out[f"{prefix}/{name}/sumsq"] = (a * a).sum().item()
            out[f"{prefix}/{name}/head"] = a[:16].numpy()
        else:
            out[f"{prefix}/{name}/int"] = t.detach().reshape(-1).numpy().astype(np.int64)
        out[f"{prefix}/{name}/shape"] = np.array(t.shape, dtype=np.int64)


def grad_norms(out, prefix, module):
    for name, p in module.named_parameters():
        if p.grad is not None:
            out[f"{prefix}/{name}"] = p.grad.detach().double().norm().item()


def seeded_uniform(shape, seed):
    g = torch.Generator().manual_seed(seed)
    return torch.rand(shape, generator=g, dtype=torch.float32)


def seeded_normal(shape, seed):
    g = torch.Generator().manual_seed(seed)
    return torch.randn(shape, generator=g, dtype=torch.float32)


# ----------------------------------------------------------------------------- goldens
def g_init(X, V, A, out_dir):
    out = {}
    torch.manual_seed(0)
    mv = V.XceptionLSTMV(128)
    state_fp(out, "V128", mv)
    out["V128/keys"] = np.array(list(mv.state_dict().keys()))
    torch.manual_seed(0)
    ma = A.XceptionLSTMA(512)
    state_fp(out, "A512", ma)
    torch.manual_seed(0)
    mx = X.xception(num_classes=1)
    state_fp(out, "X1", mx)
    np.savez_compressed(os.path.join(out_dir, "init.npz"), **out)


def g_backbone64(X, out_dir):
    """Xception backbone at 64x64 (the XceptionLSTMA frame size), train-mode BN."""
    out = {"torch_version": torch.__version__, "seed_w": 0, "seed_x": 1234, "seed_r": 99}
    torch.manual_seed(0)
    m = X.xception(num_classes=1000)
    m.fc = nn.Identity()
    m.train()
    x = seeded_uniform((4, 3, 64, 64), 1234)
    f = m(x)
    out["features"] = f.detach().numpy()
    r = seeded_normal(f.shape, 99)
    (f * r).sum().backward()
    grad_norms(out, "gradnorm", m)
    for name, t in m.state_dict().items():
        if "running" in name:
            a = t.double()
            out[f"buf/{name}/sum"] = a.sum().item()
            out[f"buf/{name}/sumsq"] = (a * a).sum().item()
    # a few full grads (small tensors) for tight checks
    out["grad/conv4.pointwise.weight/fp_sum"] = m.conv4.pointwise.weight.grad.double().sum().item()
    out["grad/conv1.weight"] = m.conv1.weight.grad.numpy()
    out["grad/block4.rep.1.conv1.weight"] = m.block4.rep[1].conv1.weight.grad.numpy()
    out["grad/bn4.weight"] = m.bn4.weight.grad.numpy()
    m.eval()
    with torch.no_grad():
        out["features_eval"] = m(x).numpy()
    np.savez_compressed(os.path.join(out_dir, "backbone64.npz"), **out)


def _logit_hook(store):
    def hook(mod, inp, outp):
        store["logits"] = outp.detach().clone()
    return hook


def g_lstmv(V, out_dir, B=2, T=4, S=299):
    """XceptionLSTMV(128) train step semantics of train_visual.py (BCE variant) at B=2,T=4,299^2."""
    out = {"torch_version": torch.__version__, "B": B, "T": T, "S": S, "seed_w": 0, "seed_x": 1234}
    x = seeded_uniform((B, T, 3, S, S), 1234)
    y = torch.tensor([[0.0], [1.0]])[:B]
    for mode in ("frozen", "unfrozen"):
        torch.manual_seed(0)
        m = V.XceptionLSTMV(128)
        if mode == "unfrozen":
            for p in m.feature_extractor.parameters():
                p.requires_grad = True
        m.train()
        m.fc_layers.eval()  # dropout off for parity (SURVEY §7 "Parity under randomness")
        store = {}
        m.fc_out.register_forward_hook(_logit_hook(store))
        feats = m.extract_features(x, "cpu")
        prob = m(feats)
        loss = nn.BCELoss()(prob, y)
        opt = torch.optim.Adam([p for p in m.parameters() if p.requires_grad], lr=1e-4)
        opt.zero_grad()
        loss.backward()
        out[f"{mode}/features"] = feats.detach().numpy()
        out[f"{mode}/prob"] = prob.detach().numpy()
        out[f"{mode}/logits"] = store["logits"].numpy()
        out[f"{mode}/loss"] = loss.item()
        grad_norms(out, f"{mode}/gradnorm", m)
        tot = torch.sqrt(sum((p.grad.double() ** 2).sum() for p in m.parameters() if p.grad is not None))
        out[f"{mode}/total_gradnorm"] = tot.item()
        opt.step()
        for name, p in m.named_parameters():
            if name.startswith("lstm.") or name.startswith("fc_out") or name in (
                    "feature_extractor.conv4.pointwise.weight", "feature_extractor.block4.rep.1.conv1.weight",
                    "feature_extractor.conv1.weight"):
                a = p.detach().double()
                out[f"{mode}/after_adam/{name}/sum"] = a.sum().item()
                out[f"{mode}/after_adam/{name}/sumsq"] = (a * a).sum().item()
        for name, t in m.state_dict().items():
            if "running_mean" in name or "running_var" in name:
                a = t.double()
                out[f"{mode}/buf/{name}/sum"] = a.sum().item()
    np.savez_compressed(os.path.join(out_dir, "lstmv_b2t4.npz"), **out)


def g_lstm(out_dir):
    out = {"torch_version": torch.__version__}
    for H, T in ((128, 16), (512, 12)):
        torch.manual_seed(0)
        lstm = nn.LSTM(2048, H, 1, batch_first=True)
        x = seeded_normal((2, T, 2048), 555).requires_grad_(True)
        o, (h, c) = lstm(x)
        r = seeded_normal(o.shape, 556)
        rh = seeded_normal(h.shape, 557)
        ((o * r).sum() + (c * rh).sum()).backward()
        p = f"H{H}"
        out[f"{p}/out"] = o.detach().numpy()
        out[f"{p}/h_n"] = h.detach().numpy()
        out[f"{p}/c_n"] = c.detach().numpy()
        out[f"{p}/dx"] = x.grad.numpy()
        for name, prm in lstm.named_parameters():
            out[f"{p}/grad/{name}"] = prm.grad.numpy() if prm.numel() <= 65536 else np.float64(
                prm.grad.double().norm().item())
            out[f"{p}/gradsum/{name}"] = prm.grad.double().sum().item()
    np.savez_compressed(os.path.join(out_dir, "lstm.npz"), **out)


def g_lstm_t120(out_dir, B=2, T=120, H=512):
    """nn.LSTM(2048, 512) over XceptionLSTMA's own recurrence length (audio_dataloader.py:20,39: 120
    MFCC frames per clip; XceptionLSTMA.py:14-19, train_audio.py:15).  Large tensors as fingerprints;
    the per-time-step norms of out pin the error growth over the 120 steps."""
    out = {"torch_version": torch.__version__, "B": B, "T": T, "H": H, "seed_w": 0, "seed_x": 555,
           "seed_r": 556, "seed_rc": 557}
    torch.manual_seed(0)
    lstm = nn.LSTM(2048, H, 1, batch_first=True)
    x = seeded_normal((B, T, 2048), 555).requires_grad_(True)
    o, (h, c) = lstm(x)
    r = seeded_normal(o.shape, 556)
    rc = seeded_normal(c.shape, 557)
    ((o * r).sum() + (c * rc).sum()).backward()
    put_fp(out, "out", o)
    out["out_step_norm"] = o.detach().double().norm(dim=2).numpy()   # [B, T]
    out["out_last"] = o.detach()[:, -1].numpy()
    out["h_n"] = h.detach().numpy()
    out["c_n"] = c.detach().numpy()
    put_fp(out, "dx", x.grad)
    out["dx_step_norm"] = x.grad.double().norm(dim=2).numpy()
    for name, prm in lstm.named_parameters():
        out[f"gradnorm/{name}"] = prm.grad.double().norm().item()
        put_fp(out, f"grad/{name}", prm.grad)
        if prm.dim() == 1:
            out[f"gradfull/{name}"] = prm.grad.numpy()
    np.savez_compressed(os.path.join(out_dir, "lstm_t120.npz"), **out)


def g_audio_t120(A, out_dir, B=2, T=120):
    """XceptionLSTMA(512) train step (train_audio.py:33-44: BCELoss on the sigmoid output, Adam 1e-4)
    at the reference's own clip length, T = 120 MFCC frames (audio_dataloader.py:20,39): 240 frames
    of 64^2 through the backbone, then H = 512 over 120 steps.  Frozen backbone (as shipped,
    XceptionLSTMA.py:11-12) and unfrozen; head dropout off."""
    out = {"torch_version": torch.__version__, "B": B, "T": T, "seed_w": 0, "seed_x": 778}
    x = seeded_normal((B, T, 3, 13), 778)
    y = torch.tensor([[1.0], [0.0]])[:B]
    for mode in ("frozen", "unfrozen"):
        torch.manual_seed(0)
        m = A.XceptionLSTMA(512)
        if mode == "unfrozen":
            for p in m.feature_extractor.parameters():
                p.requires_grad = True
        m.train()
        m.fc_layers.eval()
        store = {}
        m.fc_out.register_forward_hook(_logit_hook(store))
        feats = m.extract_features(x, "cpu")
        prob = m(feats)
        loss = nn.BCELoss()(prob, y)
        opt = torch.optim.Adam([p for p in m.parameters() if p.requires_grad], lr=1e-4)
        opt.zero_grad()
        loss.backward()
        put_fp(out, f"{mode}/features", feats)
        lo, _ = m.lstm(feats.detach())
        out[f"{mode}/lstm_last"] = lo[:, -1].detach().numpy()
        out[f"{mode}/prob"] = prob.detach().numpy()
        out[f"{mode}/logits"] = store["logits"].numpy()
        out[f"{mode}/loss"] = loss.item()
        grad_norms(out, f"{mode}/gradnorm", m)
        opt.step()
        for name, p in m.named_parameters():
            if name.startswith("lstm.") or name.startswith("fc_out"):
                a = p.detach().double()
                out[f"{mode}/after_adam/{name}/sum"] = a.sum().item()
                out[f"{mode}/after_adam/{name}/sumsq"] = (a * a).sum().item()
        for name, t in m.state_dict().items():
            if "running_mean" in name or "running_var" in name:
                out[f"{mode}/buf/{name}/sum"] = t.double().sum().item()
    np.savez_compressed(os.path.join(out_dir, "audio_b2t120.npz"), **out)


def g_blocks(X, out_dir):
    """Block fwd/bwd at N=2 in train mode: block1 (s2, no leading relu), block4 (identity skip),
    block12 (grow_first=False, s2)."""
    out = {"torch_version": torch.__version__}
    cfgs = {"block1": (64, 128, 2, 2, False, True, 37),
            "block4": (728, 728, 3, 1, True, True, 19),
            "block12": (728, 1024, 2, 2, True, False, 19)}
    for i, (name, (cin, cout, reps, s, swr, gf, hw)) in enumerate(cfgs.items()):
        torch.manual_seed(10 + i)
        blk = X.Block(cin, cout, reps, s, start_with_relu=swr, grow_first=gf)
        for mm in blk.modules():  # Xception.__init__ re-init scheme (Xception.py:154-160)
            if isinstance(mm, nn.Conv2d):
                n = mm.kernel_size[0] * mm.kernel_size[1] * mm.out_channels
                mm.weight.data.normal_(0, (2.0 / n) ** 0.5)
        blk.train()
        x = seeded_normal((2, cin, hw, hw), 100 + i).requires_grad_(True)
        y = blk(x)
        r = seeded_normal(y.shape, 200 + i)
        (y * r).sum().backward()
        put_fp(out, f"{name}/out", y)
        put_fp(out, f"{name}/dx", x.grad)
        grad_norms(out, f"{name}/gradnorm", blk)
        for bn, t in blk.state_dict().items():
            if "running" in bn:
                out[f"{name}/buf/{bn}/sum"] = t.double().sum().item()
        out[f"{name}/cfg"] = np.array([cin, cout, reps, s, int(swr), int(gf), hw])
    np.savez_compressed(os.path.join(out_dir, "blocks.npz"), **out)


def g_sepconv(X, out_dir):
    """SeparableConv2d (dw3x3 + pw1x1) per distinct backbone shape at N=2."""
    out = {"torch_version": torch.__version__}
    shapes = [(64, 128, 37), (128, 256, 37), (256, 728, 19), (728, 728, 19), (728, 1024, 19),
              (1024, 1536, 10), (1536, 2048, 10)]
    for i, (cin, cout, hw) in enumerate(shapes):
        torch.manual_seed(30 + i)
        sc = X.SeparableConv2d(cin, cout, 3, 1, 1)
        x = seeded_normal((2, cin, hw, hw), 300 + i).requires_grad_(True)
        y = sc(x)
        r = seeded_normal(y.shape, 400 + i)
        (y * r).sum().backward()
        k = f"s{cin}_{cout}_{hw}"
        put_fp(out, f"{k}/y", y)
        put_fp(out, f"{k}/dx", x.grad)
        out[f"{k}/dw_grad"] = sc.conv1.weight.grad.numpy()
        out[f"{k}/pw_gradnorm"] = sc.pointwise.weight.grad.double().norm().item()
        out[f"{k}/cfg"] = np.array([cin, cout, hw, 30 + i, 300 + i, 400 + i])
    np.savez_compressed(os.path.join(out_dir, "sepconv.npz"), **out)


def g_audio(A, out_dir, B=2, T=6):
    out = {"torch_version": torch.__version__, "B": B, "T": T}
    torch.manual_seed(0)
    m = A.XceptionLSTMA(512)
    m.train()
    m.fc_layers.eval()
    x = seeded_normal((B, T, 3, 13), 777)
    frames = F.interpolate(x.view(B * T, 3, 13, 1), size=(64, 64), mode="bilinear", align_corners=False)
    out["frames"] = frames.numpy()[:2]
    put_fp(out, "frames_fp", frames)
    store = {}
    m.fc_out.register_forward_hook(_logit_hook(store))
    feats = m.extract_features(x, "cpu")
    prob = m(feats)
    y = torch.tensor([[1.0], [0.0]])[:B]
    loss = nn.BCELoss()(prob, y)
    loss.backward()
    out["features"] = feats.detach().numpy()
    out["prob"] = prob.detach().numpy()
    out["logits"] = store["logits"].numpy()
    out["loss"] = loss.item()
    grad_norms(out, "gradnorm", m)
    np.savez_compressed(os.path.join(out_dir, "audio_b2t6.npz"), **out)


def all_param_fp(out, prefix, module):
    for name, p in module.named_parameters():
        a = p.detach().double()
        out[f"{prefix}/{name}/sum"] = a.sum().item()
        out[f"{prefix}/{name}/sumsq"] = (a * a).sum().item()


def _checkpoint_blocks(xc):
    """Recompute each Xception block in backward (torch.utils.checkpoint, non-reentrant) so a
    256-frame 299^2 step fits in the capture container's memory (the reference's autograd
    saves ~0.31 GB per frame).  The recompute runs the same CPU ops on the same inputs, so the
    gradients are those of the plain step; it re-runs the blocks' train-mode BatchNorms, so the
    running buffers are recorded before backward."""
    import torch.utils.checkpoint as cp
    for i in range(1, 13):
        blk = getattr(xc, f"block{i}")
        fwd = blk.forward
        blk.forward = (lambda f: (lambda inp: cp.checkpoint(f, inp, use_reentrant=False)))(fwd)


def g_lstmv_big(V, out_dir, B=4, T=16, S=299, labels=(0.0, 1.0, 1.0, 0.0), name="lstmv_b4t16.npz", ckpt=False):
    """The bench-size kernel set: XceptionLSTMV(128) unfrozen at B*T frames of 299^2 (B4T16:
    M = 23,104 pixel rows in the middle flow, so the 256x256 MFMA GEMMs dispatch; B16T16: the
    bench configuration itself, 256 frames, M = 92,416), one train_visual.py optimiser step:
    BCE -> backward -> clip_grad_norm_(1.0) -> Adam(lr 1e-5, weight_decay 1e-4)
    (train_visual.py:533, :575-577; BCE head as XceptionLSTMV.forward).  Stores fingerprints
    only (features, gradient norms, parameters after the step, buffers)."""
    out = {"torch_version": torch.__version__, "B": B, "T": T, "S": S, "seed_w": 0, "seed_x": 4242,
           "lr": 1e-5, "weight_decay": 1e-4, "max_norm": 1.0, "labels": np.array(labels[:B])}
    x = seeded_uniform((B, T, 3, S, S), 4242)
    y = torch.tensor([[v] for v in labels[:B]])
    torch.manual_seed(0)
    m = V.XceptionLSTMV(128)
    for p in m.feature_extractor.parameters():
        p.requires_grad = True
    m.train()
    m.fc_layers.eval()
    if ckpt:
        _checkpoint_blocks(m.feature_extractor)
    store = {}
    m.fc_out.register_forward_hook(_logit_hook(store))
    feats = m.extract_features(x, "cpu")
    del x
    prob = m(feats)
    loss = nn.BCELoss()(prob, y)
    bufs = {}
    for bname, t in m.state_dict().items():
        if "running_mean" in bname or "running_var" in bname:
            a = t.double()
            bufs[f"buf/{bname}/sum"] = a.sum().item()
            bufs[f"buf/{bname}/sumsq"] = (a * a).sum().item()
    loss.backward()
    put_fp(out, "features", feats)
    out["logits"] = store["logits"].numpy()
    out["loss"] = loss.item()
    grad_norms(out, "gradnorm", m)
    for hn, p in m.named_parameters():   # head gradients in full (small), for the bf16 head check
        if hn.startswith(("lstm.bias", "fc_out.")) and p.grad is not None:
            out[f"grad/{hn}"] = p.grad.numpy()
    params = [p for p in m.parameters() if p.requires_grad]
    out["total_gradnorm"] = torch.nn.utils.clip_grad_norm_(params, 1.0).item()
    opt = torch.optim.Adam(params, lr=1e-5, weight_decay=1e-4)
    opt.step()
    all_param_fp(out, "after_step", m)
    out.update(bufs)
    np.savez_compressed(os.path.join(out_dir, name), **out)


def g_xception_frames(X, out_dir, B, name, ckpt=False):
    """Configs C1 / C2 (BASELINE.json configs[0], [1]): xception(num_classes=1) trained per frame
    (Xception.py:205-213), B frames of 299^2, BCEWithLogitsLoss on the logits, Adam(lr 1e-5,
    weight_decay 1e-4) (the optimiser of train_visual.py:533), no clipping.  Full logits, loss,
    every gradient norm, every parameter after the step, BatchNorm buffers."""
    S = 299
    out = {"torch_version": torch.__version__, "B": B, "S": S, "seed_w": 0, "seed_x": 5151 + B,
           "lr": 1e-5, "weight_decay": 1e-4}
    x = seeded_uniform((B, 3, S, S), 5151 + B)
    y = (torch.arange(B) % 3 == 0).float().view(B, 1)
    torch.manual_seed(0)
    m = X.xception(num_classes=1)
    m.train()
    if ckpt:
        _checkpoint_blocks(m)
    logits = m(x)
    loss = nn.BCEWithLogitsLoss()(logits, y)
    bufs = {}
    for bname, t in m.state_dict().items():
        if "running_mean" in bname or "running_var" in bname:
            a = t.double()
            bufs[f"buf/{bname}/sum"] = a.sum().item()
            bufs[f"buf/{bname}/sumsq"] = (a * a).sum().item()
    loss.backward()
    out["logits"] = logits.detach().numpy()
    out["loss"] = loss.item()
    grad_norms(out, "gradnorm", m)
    out["grad/fc.weight"] = m.fc.weight.grad.numpy()
    out["grad/fc.bias"] = m.fc.bias.grad.numpy()
    out["total_gradnorm"] = torch.sqrt(sum((p.grad.double() ** 2).sum() for p in m.parameters())).item()
    opt = torch.optim.Adam(m.parameters(), lr=1e-5, weight_decay=1e-4)
    opt.step()
    all_param_fp(out, "after_step", m)
    out.update(bufs)
    np.savez_compressed(os.path.join(out_dir, name), **out)


# ----------------------------------------------------------------------------- script-level defs
def load_script_defs(fname, names, extra_globals=None):
    """Executes ONLY the named top-level class / function definitions of a reference script
    (the scripts themselves import modules absent from the snapshot, so they cannot be
    imported whole; their definitions are self-contained).  Parsed with ``ast`` from the
    read-only reference file; nothing is written there."""
    import ast
    import sklearn.metrics as skm
    src = open(os.path.join(REF, fname)).read()
    tree = ast.parse(src)
    nodes = [n for n in tree.body if isinstance(n, (ast.ClassDef, ast.FunctionDef)) and n.name in names]
    assert sorted(n.name for n in nodes) == sorted(names), (fname, [n.name for n in nodes])
    ns = {"np": np, "torch": torch, "nn": nn, "F": F, "Optional": __import__("typing").Optional,
          "roc_curve": skm.roc_curve, "roc_auc_score": skm.roc_auc_score, "auc": skm.auc, "sk_auc": skm.auc,
          "average_precision_score": skm.average_precision_score}
    ns.update(extra_globals or {})
    exec(compile(ast.Module(body=nodes, type_ignores=[]), os.path.join(REF, fname), "exec"), ns)
    return {n: ns[n] for n in names}


def metric_cases():
    """Seeded (labels, scores) sets: separable-ish, ties, heavy imbalance, and one class."""
    rs = np.random.RandomState(11)
    cases = []
    y = rs.randint(0, 2, 200)
    cases.append((y, np.clip(0.5 + 0.35 * (y - 0.5) + 0.25 * rs.randn(200), 0, 1)))
    y = rs.randint(0, 2, 64)
    cases.append((y, np.round(rs.rand(64), 1)))                       # many ties
    y = (rs.rand(300) < 0.1).astype(int)
    cases.append((y, rs.rand(300) * 0.5 + 0.4 * y))                    # 10 % positives
    cases.append((np.array([0, 1, 0, 1, 1]), np.array([0.1, 0.9, 0.8, 0.3, 0.6])))
    cases.append((np.zeros(10, int), rs.rand(10)))                     # single class
    return cases


def g_heads(out_dir):
    """Heads, losses and metrics of the training / evaluation scripts:
    ArcFaceHead (train_visual.py:455-474, m=0.5; train_au_face.py:423-442, m=0.30),
    CBFocalLoss (train_au_face.py:445-458), compute_metrics (train_visual.py:476-487,
    test_visual.py:515-565), compute_eer_auc / pick_threshold / compute_acc_ap_and_counts
    (train_au_face.py:462-506) and _unwrap_state_dict (test_au_face.py:107-125)."""
    out = {"torch_version": torch.__version__}
    tv = load_script_defs("train_visual.py", ["ArcFaceHead", "compute_metrics"])
    ta = load_script_defs("train_au_face.py", ["ArcFaceHead", "CBFocalLoss", "compute_eer_auc", "pick_threshold",
                                               "compute_acc_ap_and_counts"])
    te = load_script_defs("test_visual.py", ["compute_metrics"])
    tf = load_script_defs("test_au_face.py", ["_unwrap_state_dict"])
    for tag, cls, m_ in (("v", tv["ArcFaceHead"], 0.5), ("a", ta["ArcFaceHead"], 0.30)):
        torch.manual_seed(21)
        head = cls(128, 2, s=30.0, m=m_)
        B = 16
        f = seeded_normal((B, 128), 501).requires_grad_(True)
        lab = torch.from_numpy(np.random.RandomState(502).randint(0, 2, B)).long()
        with torch.no_grad():   # clamp edge: row 0 exactly along its class centre (cos = 1)
            f[0] = head.weight[lab[0]] * 3.0
        out[f"{tag}/weight"] = head.weight.detach().numpy()
        out[f"{tag}/features"] = f.detach().numpy()
        out[f"{tag}/labels"] = lab.numpy()
        out[f"{tag}/logits_nolabel"] = head(f).detach().numpy()
        logits = head(f, lab)
        out[f"{tag}/logits"] = logits.detach().numpy()
        if tag == "v":
            loss = nn.CrossEntropyLoss()(logits, lab)
        else:
            cb = ta["CBFocalLoss"]([300, 1700], beta=0.9999, gamma=2.0)
            out["a/class_weights"] = cb.class_weights.numpy()
            loss = cb(logits, lab)
        loss.backward()
        out[f"{tag}/loss"] = loss.item()
        out[f"{tag}/dfeatures"] = f.grad.numpy()
        out[f"{tag}/dweight"] = head.weight.grad.numpy()
    for i, (y, s) in enumerate(metric_cases()):
        out[f"m{i}/labels"] = y
        out[f"m{i}/scores"] = s
        out[f"m{i}/train_visual"] = np.array(tv["compute_metrics"](y, s), dtype=np.float64)
        r = te["compute_metrics"](y, s)
        out[f"m{i}/test_visual_keys"] = np.array(sorted(r))
        out[f"m{i}/test_visual"] = np.array([r[k] for k in sorted(r)], dtype=np.float64)
        if len(np.unique(y)) > 1:
            a_, p_, e_, _ = ta["compute_eer_auc"](y, s)
            out[f"m{i}/eer_auc"] = np.array([a_, p_, e_])
            for mode in ("youden", "fpr"):
                thr = ta["pick_threshold"](y, s, mode=mode, fpr_target=0.05)
                out[f"m{i}/thr_{mode}"] = np.array(thr)
                out[f"m{i}/acc_{mode}"] = np.array(ta["compute_acc_ap_and_counts"](y, s, thr[0]), dtype=np.float64)
    raw = {"model": {"module.conv.weight": torch.ones(2), "module.fc.bias": torch.zeros(3)}, "best_auc": 0.9,
           "n_averaged": torch.tensor(4)}
    out["unwrap/keys"] = np.array(sorted(tf["_unwrap_state_dict"](raw)))
    raw2 = {"ema_state_dict": {"n_averaged": torch.tensor(3), "module.block.w": torch.ones(1)}}
    out["unwrap2/keys"] = np.array(sorted(tf["_unwrap_state_dict"](raw2)))
    np.savez_compressed(os.path.join(out_dir, "heads.npz"), **out)


def g_arcface_step(V, out_dir, B=2, T=3):
    """The active train_visual.py step (:563-577) on CPU fp32 (autocast("cuda") and GradScaler are
    no-ops without CUDA): extract_features -> model.lstm(f)[0][:, -1] -> ArcFaceHead(128, 2, s=30,
    m=0.5) -> CrossEntropyLoss -> backward -> clip_grad_norm_(1.0) -> Adam(lr 1e-5, wd 1e-4) over
    model + head parameters, at the reference's own frame sizes 224^2 (train_visual.py:505) and
    256^2 (video_dataloader.py:61), frozen (epochs < 3) and unfrozen (train_visual.py:547-556).
    The shipped extract_features(x, seq_lengths) raises, so the device form is used."""
    tv = load_script_defs("train_visual.py", ["ArcFaceHead"])
    out = {"torch_version": torch.__version__, "B": B, "T": T}
    for S, mode in ((224, "unfrozen"), (224, "frozen"), (256, "unfrozen")):
        tag = f"s{S}_{mode}"
        torch.manual_seed(0)
        m = V.XceptionLSTMV(128)
        torch.manual_seed(1)
        head = tv["ArcFaceHead"](128, 2, s=30.0, m=0.5)
        for p in m.feature_extractor.parameters():
            p.requires_grad = mode == "unfrozen"
        m.train()
        head.train()
        x = seeded_uniform((B, T, 3, S, S), 6000 + S)
        lab = torch.tensor([0, 1])[:B]
        params = list(m.parameters()) + list(head.parameters())
        opt = torch.optim.Adam(params, lr=1e-5, weight_decay=1e-4)
        opt.zero_grad()
        feats = m.extract_features(x, "cpu")
        emb = m.lstm(feats)[0][:, -1, :]
        logits = head(emb, lab)
        loss = nn.CrossEntropyLoss()(logits, lab)
        loss.backward()
        out[f"{tag}/logits"] = logits.detach().numpy()
        out[f"{tag}/emb"] = emb.detach().numpy()
        out[f"{tag}/loss"] = loss.item()
        grad_norms(out, f"{tag}/gradnorm", m)
        out[f"{tag}/gradnorm/head.weight"] = head.weight.grad.double().norm().item()
        out[f"{tag}/total_gradnorm"] = torch.nn.utils.clip_grad_norm_(params, 1.0).item()
        opt.step()
        all_param_fp(out, f"{tag}/after_step", m)
        out[f"{tag}/after_step/head.weight"] = head.weight.detach().numpy()
    out["head_init"] = _head_init(tv, 1)
    np.savez_compressed(os.path.join(out_dir, "arcface_step.npz"), **out)


def _head_init(tv, seed):
    torch.manual_seed(seed)
    return tv["ArcFaceHead"](128, 2, s=30.0, m=0.5).weight.detach().numpy()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=os.path.join(os.path.dirname(__file__), "..", "tests", "golden"))
    ap.add_argument("--only", default="")
    args = ap.parse_args()
    os.makedirs(args.out, exist_ok=True)
    X, V, A = load_reference()
    jobs = {"init": lambda: g_init(X, V, A, args.out), "backbone64": lambda: g_backbone64(X, args.out),
            "lstm": lambda: g_lstm(args.out), "blocks": lambda: g_blocks(X, args.out),
            "sepconv": lambda: g_sepconv(X, args.out), "audio": lambda: g_audio(A, args.out),
            "lstmv": lambda: g_lstmv(V, args.out), "lstmv_big": lambda: g_lstmv_big(V, args.out),
            "lstmv_b16t16": lambda: g_lstmv_big(V, args.out, B=16, T=16, labels=tuple(float(i % 2) for i in range(16)),
                                                name="lstmv_b16t16.npz", ckpt=True),
            "c1": lambda: g_xception_frames(X, args.out, 4, "xception_c1_b4.npz"),
            "c2": lambda: g_xception_frames(X, args.out, 64, "xception_c2_b64.npz", ckpt=True),
            "heads": lambda: g_heads(args.out), "arcface_step": lambda: g_arcface_step(V, args.out),
            "lstm_t120": lambda: g_lstm_t120(args.out), "audio_t120": lambda: g_audio_t120(A, args.out)}
    for k, fn in jobs.items():
        if args.only and k not in args.only.split(","):
            continue
        print("capturing", k, flush=True)
        fn()


if __name__ == "__main__":
    main()
