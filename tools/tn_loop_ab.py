"""A/B of the 256x256 weight-gradient kernel's main loop: one 32-MFMA phase per 32-row step with
the fill four steps ahead (gemm_tn256q_kernel, XCP_TN_LOOP=2) against two 16-MFMA phases with the
fill three steps ahead (gemm_tn256_kernel).  For every step shape: the fp32 partial slabs bitwise
equal between the two (same MFMA order per accumulator), then interleaved timings of the kernel
alone (HIP events, median of rounds) at the split count the step uses.

usage: python tools/tn_loop_ab.py [rounds]
"""
import os
import statistics
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "multimodal-deepfake-detection_amd"), REPO]
from xcp import ops  # noqa: E402

SHAPES = [(1401856, 256, 256), (350464, 728, 256), (350464, 728, 728), (92416, 728, 728), (92416, 1024, 728),
          (25600, 1536, 1024), (25600, 2048, 1536), (3000, 296, 520)]


def timeit(fn, iters=10, warm=2):
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
    dev = torch.device("cuda:0")
    ops._lib.load()
    g = torch.Generator(device=dev).manual_seed(0)
    for (m, n, k) in SHAPES:
        Gt = torch.randn(m, n, device=dev, generator=g).to(torch.bfloat16)
        Xt = torch.randn(m, k, device=dev, generator=g).to(torch.bfloat16)
        rps = ops._lib.call("xcp_gemm_tn_rows_per_split", 1, 0, m, n, k, 2)
        S = (m + rps - 1) // rps
        outs = {}
        for form in ("1", "2"):
            os.environ["XCP_TN_LOOP"] = form
            P = torch.full((S * n * k,), float("nan"), device=dev)
            ops.gemm_tn(Gt, Xt, P, m, n, k, S, rps, tile=2)
            torch.cuda.synchronize()
            outs[form] = P
        ok = torch.equal(outs["1"], outs["2"])
        P = torch.empty(S * n * k, device=dev)
        t = {"1": [], "2": []}
        for _ in range(rounds):
            for form in ("1", "2"):
                os.environ["XCP_TN_LOOP"] = form
                t[form].append(timeit(lambda: ops.gemm_tn(Gt, Xt, P, m, n, k, S, rps, tile=2)))
        a, b = statistics.median(t["1"]), statistics.median(t["2"])
        fl = 2.0 * m * n * k
        print(f"{m:8d}x{n:5d}x{k:5d} S={S:3d}  2-phase {a:8.1f} us  1-phase {b:8.1f} us  ({(b / a - 1) * 100:+5.1f} %, "
              f"{fl / b / 1e6:6.0f} TFLOP/s)  bitwise {ok}", flush=True)
        del Gt, Xt, P, outs
    os.environ.pop("XCP_TN_LOOP", None)


if __name__ == "__main__":
    main()
