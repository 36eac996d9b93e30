"""Stem conv2 forward (+BN partial sums) at 256 frames of 149^2 x 32 -> 147^2 x 64: one 8-wave workgroup
per CU on 4-row tiles vs two 4-wave workgroups per CU on 2-row tiles (XCP_CONV3_FWD_2WG, read per call),
interleaved rounds, median, HIP events.

  python tools/conv3_ab.py      # GPU box
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
    N = 256
    a1 = torch.randn(N * 149 * 149, 32, device=dev, generator=g).bfloat16()
    w2 = (torch.randn(64, 288, device=dev, generator=g) / 17).bfloat16()
    c2 = torch.empty(N * 147 * 147, 64, device=dev, dtype=torch.bfloat16)
    st = torch.empty(2 * 256 * 2 * 64, device=dev)
    times = {"0": [], "1": []}
    for _ in range(5):
        for v in times:
            os.environ["XCP_CONV3_FWD_2WG"] = v
            for _w in range(2):
                ops.conv3x3(0, a1, w2, c2, st, N, 149, 149)
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            for _i in range(10):
                ops.conv3x3(0, a1, w2, c2, st, N, 149, 149)
            e.record()
            torch.cuda.synchronize()
            times[v].append(s.elapsed_time(e) / 10 * 1e3)
    byts = (a1.numel() + c2.numel()) * 2
    for v, t in times.items():
        m = statistics.median(t)
        print(f"XCP_CONV3_FWD_2WG={v}: {m:7.1f} us  {byts / m / 1e3:6.0f} GB/s  (rounds " + " ".join(f"{x:.1f}" for x in t) + ")",
              flush=True)
    os.environ.pop("XCP_CONV3_FWD_2WG", None)


if __name__ == "__main__":
    main()
