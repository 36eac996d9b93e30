"""A/B of the H = 512 LSTM recurrence: the per-step kernels (120 launches per direction) against the
persistent kernels (one launch per direction), forward and backward timed separately with HIP
events at XceptionLSTMA's shape (B = 16 clips, T = 120, H = 512), at B = 2 and at H = 256.

usage: python tools/lstm_ab.py [rounds]
"""
import os
import statistics
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "multimodal-deepfake-detection_amd"), REPO]
from xcp import ops  # noqa: E402


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
    for (B, T, H) in ((16, 120, 512), (2, 120, 512), (8, 120, 256)):
        G4 = 4 * H
        xp = torch.randn(B, T, G4, device=dev, generator=g)
        whh = torch.randn(G4, H, device=dev, generator=g) / H ** 0.5
        bih, bhh = torch.zeros(G4, device=dev), torch.zeros(G4, device=dev)
        out, hp, cs = (torch.empty(B, T, H, device=dev) for _ in range(3))
        gt = torch.empty(B, T, G4, device=dev)
        hn, cn = torch.empty(B, H, device=dev), torch.empty(B, H, device=dev)
        dout = torch.randn(B, T, H, device=dev, generator=g)
        dg = torch.empty(B, T, G4, device=dev)
        fwd = lambda: ops.lstm_fwd(xp, whh, None, bih, bhh, out, hp, cs, gt, hn, cn, B, T, H)   # noqa: E731
        bwd = lambda: ops.lstm_bwd(dout, None, None, whh, cs, gt, dg, B, T, H)   # noqa: E731
        # per-step kernels, persistent (backward: dh partials), persistent (backward: gather), (backward: clip-grouped gather)
        forms = ("0", "1", "g", "c", "c2")
        t = {(f, d): [] for f in forms for d in ("fwd", "bwd")}
        for _ in range(rounds):
            for form in forms:
                os.environ["XCP_LSTM_PERSIST"] = "0" if form == "0" else "1"
                os.environ["XCP_LSTM_BWD"] = {"g": "gather", "c": "cg", "c2": "cg2"}.get(form, "partials")
                t[(form, "fwd")].append(timeit(fwd))
                t[(form, "bwd")].append(timeit(bwd))
        err = ops.lstm_sync_error()
        for d in ("fwd", "bwd"):
            a, b, c, cg, cg2 = (statistics.median(t[(f, d)]) for f in forms)
            print(f"B={B:2d} T={T} H={H} {d}: per-step {a:8.1f} us ({a / T:5.2f} us/step)  persistent {b:8.1f} us "
                  f"({b / T:5.2f} us/step, {(b / a - 1) * 100:+6.1f} %)" +
                  (f"  gather {c:8.1f} us ({c / T:5.2f} us/step, {(c / a - 1) * 100:+6.1f} %)"
                   f"  clip-grouped {cg:8.1f} us ({cg / T:5.2f} us/step, {(cg / a - 1) * 100:+6.1f} %)"
                   f"  cg2 {cg2:8.1f} us ({cg2 / T:5.2f} us/step, {(cg2 / a - 1) * 100:+6.1f} %)" if d == "bwd" else "") +
                  f"  sync_error={err}", flush=True)
    os.environ.pop("XCP_LSTM_PERSIST", None)
    os.environ.pop("XCP_LSTM_BWD", None)


if __name__ == "__main__":
    main()
