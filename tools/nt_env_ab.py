"""A/B of two forms of the persistent 256x256 NT kernel selected by an environment variable the
library reads per call (e.g. XCP_NT_PF2=0,1: the two-K-tile prefetch at tile boundaries).  For every
shape: C bitwise equal between the two, BN statistics equal to fp32 rounding, then interleaved timings
(HIP events, median of rounds).

usage: python tools/nt_env_ab.py [rounds] [VAR=a,b]
"""
import os
import statistics
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "multimodal-deepfake-detection_amd"), REPO]
from xcp import ops  # noqa: E402

SHAPES = [  # (M, N, K, stats, tile) -- the step's persistent-kernel calls, and whole rounds of 256 tiles
    (92416, 736, 736, True, 0), (92416, 736, 736, False, 0), (350464, 736, 736, True, 0),
    (350464, 736, 256, True, 0), (350464, 256, 736, False, 0), (1401856, 256, 256, True, 0),
    (1401856, 256, 128, True, 0), (92416, 1024, 736, True, 0), (92416, 736, 1024, False, 0),
    (25600, 1536, 1024, True, 0), (25600, 2048, 1536, True, 0), (25600, 1024, 1536, False, 0),
    (65536, 1024, 768, False, 3), (65536, 1024, 3072, False, 3), (1000, 520, 200, True, 3),
    (350464, 256, 128, False, 0), (350464, 512, 128, True, 0), (65536, 1024, 64, False, 3),
    (65536, 1024, 128, True, 3), (30720, 736, 736, True, 0),
]


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
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    var, vals = (sys.argv[2] if len(sys.argv) > 2 else "XCP_NT_PF2=0,1").split("=")
    fa, fb = vals.split(",")
    dev = torch.device("cuda:0")
    ops._lib.load()
    g = torch.Generator(device=dev).manual_seed(0)
    for (m, n, k, stats, tile) in SHAPES:
        X = torch.randn(m, k, device=dev, generator=g).to(torch.bfloat16)
        Wt = (torch.randn(n, k, device=dev, generator=g) / 27).to(torch.bfloat16)
        outs = {}
        for form in (fa, fb):
            os.environ[var] = form
            Y = torch.full((m, n), float("nan"), device=dev, dtype=torch.bfloat16)
            st = torch.full((ops.nt_stat_rows(m) * 2 * n,), float("nan"), device=dev) if stats else None
            ops.gemm_nt(X, Wt, Y, m, n, k, stats=st, tile=tile)
            torch.cuda.synchronize()
            outs[form] = (Y, st)
        Y4, s4 = outs[fa]
        Y2, s2 = outs[fb]
        ok = torch.equal(Y4, Y2) and not torch.isnan(Y2.float()).any().item()
        serr = 0.0
        if stats:
            serr = ((s2 - s4).abs().max() / s4.abs().max().clamp_min(1e-30)).item()
            ok = ok and serr < 1e-5
        Y = torch.empty(m, n, device=dev, dtype=torch.bfloat16)
        st = torch.empty(ops.nt_stat_rows(m) * 2 * n, device=dev) if stats else None
        t = {fa: [], fb: []}
        for _ in range(rounds):
            for form in (fa, fb):
                os.environ[var] = form
                t[form].append(timeit(lambda: ops.gemm_nt(X, Wt, Y, m, n, k, stats=st, tile=tile)))
        a, b = statistics.median(t[fa]), statistics.median(t[fb])
        fl = 2.0 * m * n * k
        print(f"{m:8d}x{n:5d}x{k:5d} stats={int(stats)} tile={tile}  {var}={fa} {a:8.1f} us  ={fb} {b:8.1f} us  "
              f"({(b / a - 1) * 100:+5.1f} %, {fl / b / 1e6:6.0f} TFLOP/s)  C bitwise {ok} stats rel {serr:.1e}",
              flush=True)
        del X, Wt, Y, st, outs
    os.environ.pop(var, None)


if __name__ == "__main__":
    main()
