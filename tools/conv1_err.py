"""conv1.weight's bf16 gradient-norm error on the backbone64 golden (tests/golden/backbone64.npz, 4 frames
of 64^2) for three input scales (bf16_contract.XSCALES), under the current XCP_* switches / XCP_LIB_PATH:
isolates which stem path moves it.  Prints one line.

  python tools/conv1_err.py      # GPU box
"""
import os
import sys

import numpy as np
import torch
import torch.nn as nn

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "multimodal-deepfake-detection_amd"), REPO, os.path.join(REPO, "tests")]

import bf16_contract  # noqa: E402


def main():
    import xcp
    from Models.Xception import xception
    g = np.load(os.path.join(REPO, "tests", "golden", "backbone64.npz"))
    dev = torch.device("cuda:0")
    torch.manual_seed(0)
    m = xception(num_classes=1000)
    m.fc = nn.Identity()
    m = m.to(dev).train()
    sd0 = {k: v.detach().clone() for k, v in m.state_dict().items()}
    gen = torch.Generator().manual_seed(1234)
    x = torch.rand((4, 3, 64, 64), generator=gen).to(dev)
    r = torch.randn((4, 2048), generator=torch.Generator().manual_seed(99)).to(dev)
    names = ["conv1.weight", "bn1.weight", "bn1.bias", "conv2.weight", "bn2.weight"]
    out = {n: [] for n in names}
    for c in bf16_contract.XSCALES:
        sd = dict(sd0)
        sd["conv1.weight"] = sd0["conv1.weight"] / c
        m.load_state_dict(sd)
        m.zero_grad(set_to_none=True)
        with xcp.precision("bf16"):
            (m(x * c) * r).sum().backward()
        torch.cuda.synchronize()
        p = dict(m.named_parameters())
        for n in names:
            ref = float(g[f"gradnorm/{n}"])
            gr = p[n].grad / c if n == "conv1.weight" else p[n].grad   # (the leaf is conv1.weight / c)
            out[n].append(abs(gr.double().norm().item() - ref) / ref)
    tag = " ".join(f"{k}={os.environ[k]}" for k in sorted(os.environ) if k.startswith("XCP_"))
    print(f"[{tag or 'default'}] " + "  ".join(f"{n}: " + " ".join(f"{e:.4f}" for e in v) for n, v in out.items()),
          flush=True)


if __name__ == "__main__":
    main()
