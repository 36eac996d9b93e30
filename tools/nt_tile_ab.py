"""The middle-flow pointwise op (and neighbours) on each NT kernel choice: tile 0 (automatic: persistent 256x256 +
sparse last round on 128x128), 1 (128x128 for every row), 2 (one-shot 256x256 for every row), 3 (persistent for
every row); HIP events, median of rounds.

usage: python tools/nt_tile_ab.py [rounds]
"""
import os
import statistics
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "multimodal-deepfake-detection_amd"), REPO]
from xcp import ops  # noqa: E402
from nt_env_ab import timeit  # noqa: E402

SHAPES = [(92416, 736, 736, True), (92416, 736, 736, False), (350464, 736, 736, True), (30720, 736, 736, True),
          (350464, 256, 736, False), (92416, 1024, 736, True)]


def main():
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(0)
    for (m, n, k, stats) in SHAPES:
        X = torch.randn(m, k, device=dev, generator=g).to(torch.bfloat16)
        Wt = (torch.randn(n, k, device=dev, generator=g) / 27).to(torch.bfloat16)
        Y = torch.empty(m, n, device=dev, dtype=torch.bfloat16)
        st = torch.empty(ops.nt_stat_rows(m) * 2 * n, device=dev) if stats else None
        t = {tl: [] for tl in (0, 1, 2, 3)}
        for _ in range(rounds):
            for tl in t:
                t[tl].append(timeit(lambda: ops.gemm_nt(X, Wt, Y, m, n, k, stats=st, tile=tl)))
        fl = 2.0 * m * n * k
        print(f"{m:8d}x{n:5d}x{k:5d} stats={int(stats)}  " + "  ".join(
            f"tile{tl} {statistics.median(v):7.1f} us ({fl / statistics.median(v) / 1e6:5.0f} TF)" for tl, v in t.items()),
            flush=True)
        del X, Wt, Y, st


if __name__ == "__main__":
    main()
