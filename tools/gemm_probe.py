"""NT256 fixed-cost probe: per-round time of the 256x256 NT kernel (tile=2) at K = 736 with 8-256
tiles in flight (one round, every tile on its own CU), with and without the BN-statistics
epilogue, and at K = 64 (fixed cost dominates).  Separates per-tile fixed cost under store
contention (all CUs writing their tiles at once) from the uncontended cost.

usage (GPU box): python tools/gemm_probe.py [tile ...]   (default 2)
"""
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "multimodal-deepfake-detection_amd"), REPO]
from xcp import ops  # noqa: E402


def timeit(fn, iters=30, warm=5):
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e3


def main():
    dev = torch.device("cuda:0")
    ops._lib.load()
    g = torch.Generator(device=dev).manual_seed(0)
    N = 256
    tiles_arg = [int(t) for t in sys.argv[1:]] or [2]
    for tile, K in [(t, k) for k in (736, 64) for t in tiles_arg]:
        for tiles in (8, 32, 64, 128, 256, 512, 1024):
            M = tiles * 256
            A = torch.randn(M, K, device=dev, generator=g).bfloat16()
            B = (torch.randn(N, K, device=dev, generator=g) / K ** 0.5).bfloat16()
            C = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
            st = torch.empty(ops.nt_stat_rows(M) * 2 * N, device=dev)
            t0 = timeit(lambda: ops.gemm_nt(A, B, C, M, N, K, tile=tile))
            t1 = timeit(lambda: ops.gemm_nt(A, B, C, M, N, K, stats=st, tile=tile))
            fl = 2.0 * M * N * K
            print(f"tile={tile} K={K:4d} tiles={tiles:5d}  nostats {t0:8.1f} us  stats {t1:8.1f} us   "
                  f"{fl / t0 / 1e6:7.1f} TF/s  rounds={max(1, tiles / 256):.2f}  us/round {t0 / max(1, tiles / 256):7.1f}",
                  flush=True)
            del A, B, C, st


if __name__ == "__main__":
    main()
