"""Weight-gradient GEMM (gemm_tn256_kernel) at the middle-flow shape (92,416 x 728 x 728, 736 pitch,
bf16): split counts x the XCD map of the splits (XCP_TN_XCD_ALIGN), kernel only, HIP events on the
launch stream, interleaved rounds, median.  Grids: S = 14 -> 126 (default map) / 144 (whole splits
per XCD), S = 28 -> 252 / 288, so the PMC passes (rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE over
`python tools/tn_align.py pmc`) separate the four variants by grid.

  python tools/tn_align.py [time|pmc]      # GPU box
"""
import os
import statistics
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "multimodal-deepfake-detection_amd"), REPO]

from xcp import ops  # noqa: E402


def main():
    mode = sys.argv[1] if len(sys.argv) > 1 else "time"
    dev = torch.device("cuda:0")
    ops._lib.load()
    g = torch.Generator(device=dev).manual_seed(0)
    M, C, CP = 92416, 728, 736
    G = torch.zeros(M, CP, device=dev, dtype=torch.bfloat16)
    X = torch.zeros(M, CP, device=dev, dtype=torch.bfloat16)
    G[:, :C] = torch.randn(M, C, device=dev, generator=g).bfloat16()
    X[:, :C] = torch.randn(M, C, device=dev, generator=g).bfloat16()
    variants = [(14, "0"), (14, "1"), (28, "0"), (28, "1")]
    P = torch.empty(28 * C * C, device=dev)

    def call(S, al):
        os.environ["XCP_TN_XCD_ALIGN"] = al
        rps = -(-M // S)
        rps = -(-rps // 64) * 64
        ops.gemm_tn(G, X, P, M, C, C, S, rps, ldg=CP, ldx=CP)

    if mode == "pmc":
        for v in variants:
            for _ in range(5):
                call(*v)
        torch.cuda.synchronize()
        return
    times = {v: [] for v in variants}
    for _ in range(5):
        for v in variants:
            for _w in range(2):
                call(*v)
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            for _i in range(10):
                call(*v)
            e.record()
            torch.cuda.synchronize()
            times[v].append(s.elapsed_time(e) / 10 * 1e3)
    fl = 2.0 * M * C * C
    for v, t in times.items():
        m = statistics.median(t)
        print(f"S={v[0]:3d} xcd_align={v[1]}: {m:7.1f} us  {fl / m / 1e6:7.1f} TFLOP/s  (rounds: "
              + " ".join(f"{x:.1f}" for x in t) + ")", flush=True)
    os.environ.pop("XCP_TN_XCD_ALIGN", None)


if __name__ == "__main__":
    main()
