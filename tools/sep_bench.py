"""Block1's fused depthwise + pointwise forward (xcp_sep_fwd) against the two kernels it replaces
(xcp_dw_fwd + the 128x128 NT GEMM with BN statistics), 256 frames of 147^2, bf16, BN + ReLU on load:
us per launch and the HBM rate of each form's algorithmic bytes.

usage (GPU box): python tools/sep_bench.py [iters]
"""
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "multimodal-deepfake-detection_amd"), REPO, os.path.join(REPO, "tools")]
from xcp import ops  # noqa: E402
from gemm_ab import timeit  # noqa: E402


def main():
    iters = int(sys.argv[1]) if len(sys.argv) > 1 else 10
    dev = torch.device("cuda:0")
    ops._lib.load()
    g = torch.Generator(device=dev).manual_seed(0)
    N, H, W = 256, 147, 147
    M = N * H * W
    for CIN in (64, 128):
        X = torch.randn(M, CIN, device=dev, generator=g).bfloat16()
        sc = torch.rand(CIN, device=dev, generator=g) + 0.5
        sh = torch.randn(CIN, device=dev, generator=g) * 0.5
        dwt = torch.randn(9, CIN, device=dev, generator=g) * 0.3
        pw = (torch.randn(128, CIN, device=dev, generator=g) / CIN ** 0.5).bfloat16()
        D = torch.empty(M, CIN, device=dev, dtype=torch.bfloat16)
        Y = torch.empty(M, 128, device=dev, dtype=torch.bfloat16)
        R = ops.sep_fwd_parts(torch.bfloat16, N, H, W, CIN, 128)
        part = torch.empty(R * 2 * 128, device=dev)
        Rn = ops.nt_stat_rows(M)
        partn = torch.empty(Rn * 2 * 128, device=dev)
        fused = timeit(lambda: ops.sep_fwd(2, X, sc, sh, dwt, pw, D, Y, part, N, H, W, CIN, 128), iters)
        dw = timeit(lambda: ops.dw_fwd(2, X, D, dwt, sc, sh, N, H, W, CIN), iters)
        nt = timeit(lambda: ops.gemm_nt(D, pw, Y, M, 128, CIN, stats=partn), iters)
        bf = M * (2 * CIN * 2 + 256)
        bu = M * (3 * CIN * 2 + 256)
        print(f"CIN {CIN:3d}: fused {fused:7.1f} us ({bf / fused / 1e6:5.2f} TB/s of {bf / 1e9:.2f} GB)   "
              f"dw {dw:6.1f} + NT {nt:6.1f} = {dw + nt:7.1f} us ({bu / (dw + nt) / 1e6:5.2f} TB/s of {bu / 1e9:.2f} GB)",
              flush=True)


if __name__ == "__main__":
    main()
