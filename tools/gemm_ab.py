"""Interleaved A/B of the NT GEMM variants at the middle-flow shape (M = 256 frames x 19 x 19,
736-channel pitch, bf16): tile 0 (automatic: one-shot 256x256 + sparse round on 128x128),
tile 2 (one-shot 256x256 for every row), tile 3 (persistent 256x256 + sparse round; tile 0 is now this), tile 4 (the automatic choice with the one-shot kernel), with and
without the BN-statistics epilogue.  Rounds alternate variants in one process (rule 24).

usage (GPU box): python tools/gemm_ab.py [rounds]
"""
import os
import statistics
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "multimodal-deepfake-detection_amd"), REPO]
from xcp import ops  # noqa: E402


def timeit(fn, iters=20, warm=3):
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
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 5
    dev = torch.device("cuda:0")
    ops._lib.load()
    g = torch.Generator(device=dev).manual_seed(0)
    M, N, K = 256 * 361, 736, 736
    A = torch.randn(M, K, device=dev, generator=g).bfloat16()
    B = (torch.randn(N, K, device=dev, generator=g) / K ** 0.5).bfloat16()
    C = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
    st = torch.empty(ops.nt_stat_rows(M) * 2 * N, device=dev)
    fl = 2.0 * M * 728 * 728
    variants = {f"tile{t}{'+stats' if s else ''}": (t, s) for t in (0, 4, 2, 3) for s in (True, False)}
    res = {k: [] for k in variants}
    for _ in range(rounds):
        for k, (t, s) in variants.items():
            res[k].append(timeit(lambda: ops.gemm_nt(A, B, C, M, N, K, stats=st if s else None, tile=t)))
    for k, v in res.items():
        med = statistics.median(v)
        print(f"{k:14s} median {med:7.1f} us  min {min(v):7.1f}  {fl / med / 1e6:7.1f} TF/s (728^2 flops)  "
              f"frac {fl / med / 1e6 / 2500:.3f}", flush=True)


if __name__ == "__main__":
    main()
