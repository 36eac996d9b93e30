"""Diagnostic: per-parameter gradient-norm errors of the frozen bf16 XceptionLSTMV step
against the reference goldens, under several depthwise-forward kernel choices."""
import os
import sys

import numpy as np
import torch
import torch.nn as nn

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "multimodal-deepfake-detection_amd"), REPO]
import xcp  # noqa: E402
from xcp import _lib  # noqa: E402
from Models.XceptionLSTMV import XceptionLSTMV  # noqa: E402

g = dict(np.load(os.path.join(REPO, "tests", "golden", "lstmv_b2t4.npz"), allow_pickle=False))
B, T, S = int(g["B"]), int(g["T"]), int(g["S"])
gpu = torch.device("cuda:0")
xcp.load_library()
for fam in (1, 0, 2):
    old = _lib.call("xcp_tune", 4, fam)
    torch.manual_seed(0)
    m = XceptionLSTMV(128, pretrained=False).to(gpu).train()
    m.fc_layers.eval()
    x = torch.rand((B, T, 3, S, S), generator=torch.Generator().manual_seed(1234)).to(gpu)
    y = torch.tensor([[0.0], [1.0]], device=gpu)[:B]
    with xcp.precision("bf16"):
        feats = m.extract_features(x, gpu)
        prob = m(feats)
        loss = nn.BCELoss()(prob, y)
        loss.backward()
    torch.cuda.synchronize()
    errs = {n: abs(p.grad.double().norm().item() - g[f"frozen/gradnorm/{n}"]) / g[f"frozen/gradnorm/{n}"]
            for n, p in m.named_parameters() if p.grad is not None}
    f = feats.detach().cpu().double().numpy().ravel()
    r = g["frozen/features"].ravel()
    cosv = f @ r / np.linalg.norm(f) / np.linalg.norm(r)
    print(f"fam={fam} loss={loss.item():.6f} ref={float(g['frozen/loss']):.6f} cos={cosv:.6f} "
          f"median={np.median(list(errs.values())):.4f} max={max(errs.values()):.4f}", flush=True)
    _lib.call("xcp_tune", 4, old)
