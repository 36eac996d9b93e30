"""Debug: gemm_nt4w_kernel (XCP_NT_4W=1) against gemm_nt256p_kernel on one shape: C and the BN partial rows,
where they differ (rows / columns / NaN)."""
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "multimodal-deepfake-detection_amd"), REPO]
from xcp import ops  # noqa: E402


def main():
    M, N, K = [int(v) for v in (sys.argv[1:4] if len(sys.argv) > 3 else (92416, 736, 736))]
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(M + N + K)
    A = torch.randn(M, K, device=dev, generator=g).bfloat16()
    B = (torch.randn(N, K, device=dev, generator=g) / K ** 0.5).bfloat16()
    R = ops.nt_stat_rows(M)
    outs = {}
    for form, tile in (("0", 2), ("0", 0), ("1", 0), ("1", 0), ("1", 0)):
        os.environ["XCP_NT_4W"] = form
        C = torch.full((M, N), float("nan"), device=dev, dtype=torch.bfloat16)
        part = torch.full((R, 2, N), float("nan"), device=dev)
        ops.gemm_nt(A, B, C, M, N, K, stats=part, tile=tile)
        torch.cuda.synchronize()
        outs[len(outs)] = (C, part)
    for k in range(1, len(outs)):
        print("run", k, "C equal to one-shot", torch.equal(outs[0][0], outs[k][0]), "stats equal",
              torch.equal(outs[0][1], outs[k][1]))
    C0, p0 = outs[1]
    C1, p1 = outs[2]
    print("C equal", torch.equal(C0, C1), "C nan", torch.isnan(C1.float()).sum().item())
    print("stats nan 256p", torch.isnan(p0).sum().item(), "4w", torch.isnan(p1).sum().item())
    d = (p0 - p1).abs()
    bad = (d > 0) | torch.isnan(p1)
    print("stats differing entries", bad.sum().item(), "of", p0.numel())
    idx = bad.nonzero()
    if len(idx):
        rows = idx[:, 0].unique()
        cols = idx[:, 2].unique()
        print("rows", rows[:20].tolist(), "...", len(rows), "cols", cols[:40].tolist(), "...", len(cols))
        print("which", idx[:, 1].unique().tolist())
        r, w, c = idx[0].tolist()
        print("first", r, w, c, p0[r, w, c].item(), p1[r, w, c].item())
        print("max rel", (d[~torch.isnan(d)] / p0.abs()[~torch.isnan(d)].clamp_min(1e-30)).max().item())


if __name__ == "__main__":
    main()
