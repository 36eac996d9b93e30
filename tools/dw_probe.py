"""Diagnostic: run the middle-flow depthwise forward / backward a few times (for rocprofv3
PMC passes).  usage: python tools/dw_probe.py [fwd|bwd] [iters]"""
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "multimodal-deepfake-detection_amd"), REPO]
from xcp import ops  # noqa: E402


def main():
    which = sys.argv[1] if len(sys.argv) > 1 else "bwd"
    iters = int(sys.argv[2]) if len(sys.argv) > 2 else 5
    dev = torch.device("cuda:0")
    ops._lib.load()
    N, H, W, C = 256, 19, 19, 728
    g = torch.Generator(device=dev).manual_seed(0)
    X = torch.randn(N * H * W, C, device=dev, generator=g).bfloat16()
    D = torch.randn(N * H * W, C, device=dev, generator=g).bfloat16()
    Y = torch.empty_like(X)
    Wt = torch.randn(9 * C, device=dev, generator=g) / 3
    sc, sh = torch.rand(C, device=dev) + 0.5, torch.randn(C, device=dev) * 0.1
    st = {"mean": torch.zeros(C, device=dev), "invstd": torch.ones(C, device=dev)}
    dW = torch.empty(9 * C, device=dev)
    for _ in range(iters):
        if which == "fwd":
            ops.dw_fwd(2, X, Y, Wt, sc, sh, N, H, W, C)
        else:
            ops.dw_bwd(2, D, X, Wt, sc, sh, Y, dW, N, H, W, C, bn_stats=st)
    torch.cuda.synchronize()


if __name__ == "__main__":
    main()
