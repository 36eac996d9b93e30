"""Fused block1 forward (engine.SEP_FUSED) against the two-kernel path on the same model and input:
the 64^2 backbone of test_backbone64_vs_reference (bf16) -- features of both paths, their cosine to
each other and to the reference's golden features, and the BN1-of-block1 statistics of both.

usage (GPU box): python tools/sep_diag.py
"""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "multimodal-deepfake-detection_amd"), REPO, os.path.join(REPO, "tests")]


def main():
    import torch
    import torch.nn as nn
    import xcp
    from xcp import engine
    from Models.Xception import xception
    from test_gpu_model import seeded_uniform, cos
    dev = torch.device("cuda:0")
    xcp.load_library()
    g = np.load(os.path.join(REPO, "tests", "golden", "backbone64.npz"))
    feats, bufs = {}, {}
    for fused in (False, True, False, True):
        engine.SEP_FUSED = fused
        torch.manual_seed(0)
        m = xception(num_classes=1000)
        m.fc = nn.Identity()
        m = m.to(dev).train()
        x = seeded_uniform((4, 3, 64, 64), 1234).to(dev)
        with xcp.precision("bf16"):
            f = m(x)
        torch.cuda.synchronize()
        feats.setdefault(fused, []).append(f.detach().cpu().numpy())
        bufs.setdefault(fused, []).append({n: b.detach().cpu().numpy().copy() for n, b in m.named_buffers()
                                           if "block1.rep" in n and "running" in n})
    for fused in (False, True):
        a, b = feats[fused]
        print(f"fused={fused}: run-to-run identical {np.array_equal(a, b)}; cos to golden {cos(a, g['features']):.6f}")
    print(f"cos(fused, unfused) {cos(feats[True][0], feats[False][0]):.7f}; max rel diff "
          f"{np.abs(feats[True][0] - feats[False][0]).max() / np.abs(feats[False][0]).max():.3e}")
    for n in bufs[False][0]:
        a, b = bufs[False][0][n], bufs[True][0][n]
        print(f"{n:40s} max rel diff {np.abs(a - b).max() / max(np.abs(a).max(), 1e-30):.3e}")
    # the same bf16 model under other summation orders of the BN statistics, each as valid as the
    # shipped one: the cosine to the fp32 reference's features moves by about this much
    from xcp import ops
    variants = {
        "two kernels (shipped before)": dict(SEP_FUSED=False),
        "fused": dict(SEP_FUSED=True),
        "two kernels, NT 128-tile everywhere": dict(SEP_FUSED=False, NT_TILE=1),
        "two kernels, NT one-shot 256": dict(SEP_FUSED=False, NT_TILE=2),
        "two kernels, stats pre-reduced to 3 groups": dict(SEP_FUSED=False, FIN=(1, 3)),
        "fused, stats pre-reduced to 3 groups": dict(SEP_FUSED=True, FIN=(1, 3)),
        "two kernels, stats pre-reduced to 7 groups": dict(SEP_FUSED=False, FIN=(1, 7)),
    }
    base = (engine.SEP_FUSED, engine.NT_TILE, ops.FIN_MAX_ROWS, ops.FIN_GROUPS)
    for name, v in variants.items():
        engine.SEP_FUSED = v.get("SEP_FUSED", base[0])
        engine.NT_TILE = v.get("NT_TILE", base[1])
        ops.FIN_MAX_ROWS, ops.FIN_GROUPS = v.get("FIN", (base[2], base[3]))
        torch.manual_seed(0)
        m = xception(num_classes=1000)
        m.fc = nn.Identity()
        m = m.to(dev).train()
        x = seeded_uniform((4, 3, 64, 64), 1234).to(dev)
        with xcp.precision("bf16"):
            f = m(x).detach().cpu().numpy()
        # the test's running-mean check: |sum - golden| against atol + rtol |golden| (0.05 each)
        worst, wn = 0.0, ""
        for bn, t in m.state_dict().items():
            if "running_mean" in bn:
                gs = float(g[f"buf/{bn}/sum"])
                v = abs(t.double().sum().item() - gs) / (0.05 + 0.05 * abs(gs))
                if v > worst:
                    worst, wn = v, bn
        print(f"{name:45s} cos to golden {cos(f, g['features']):.6f}   worst running_mean sum / tolerance "
              f"{worst:.2f} ({wn})")
    engine.SEP_FUSED, engine.NT_TILE, ops.FIN_MAX_ROWS, ops.FIN_GROUPS = base


if __name__ == "__main__":
    main()
