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
            "lstmv": lambda: g_lstmv(V, args.out)}
    for k, fn in jobs.items():
        if args.only and k not in args.only.split(","):
            continue
        print("capturing", k, flush=True)
        fn()


if __name__ == "__main__":
    main()
