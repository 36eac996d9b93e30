"""Depthwise forward variants read per call (XCP_DW_FWD_P: 0 = tile kernel, 2 / 4 = persistent
double-buffered with 2 / 4 workgroups per CU) at the step's shapes (256 frames, bf16, BN + ReLU on
load), interleaved rounds, median; HIP events on the launch stream; algorithmic bytes = input +
output once.

  python tools/dw_fwd_ab.py      # GPU box
"""
import os
import statistics
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "multimodal-deepfake-detection_amd"), REPO]

from xcp import ops  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    ops._lib.load()
    g = torch.Generator(device=dev).manual_seed(0)
    for N, H, C in [(256, 19, 736), (256, 37, 736), (256, 74, 256), (256, 147, 128), (256, 147, 64)]:
        W = H
        M = N * H * W
        x = torch.randn(M, C, device=dev, generator=g).bfloat16()
        y = torch.empty_like(x)
        Wt = torch.randn(9, C, device=dev, generator=g) / 3
        sc = torch.rand(C, device=dev, generator=g) + 0.5
        sh = torch.randn(C, device=dev, generator=g) * 0.2
        times = {v: [] for v in ("0", "2", "4")}
        for _ in range(5):
            for v in times:
                os.environ["XCP_DW_FWD_P"] = v
                for _ in range(2):
                    ops.dw_fwd(2, x, y, Wt, sc, sh, N, H, W, C)
                s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                s.record()
                for _ in range(10):
                    ops.dw_fwd(2, x, y, Wt, sc, sh, N, H, W, C)
                e.record()
                torch.cuda.synchronize()
                times[v].append(s.elapsed_time(e) / 10 * 1e3)
        byts = 2 * M * C * 2
        line = "  ".join(f"P={v}: {statistics.median(t):7.1f} us {byts / statistics.median(t) / 1e6:6.2f} TB/s"
                         for v, t in times.items())
        print(f"{N}x{H}^2x{C}: {line}", flush=True)
        del x, y
    os.environ.pop("XCP_DW_FWD_P", None)


if __name__ == "__main__":
    main()
