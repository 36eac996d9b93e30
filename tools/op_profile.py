"""Per-call profile of the xcp C-ABI entry points inside the bench's train step.

Wraps ``xcp._lib.call`` so every compute entry point is bracketed by HIP events on the
current stream, runs a few bench steps and prints, per (entry point, integer arguments),
the call count per step and the mean time -- the shape-level view the kernel-trace
summary cannot give (it only knows grid sizes).  Diagnostic only.

usage: python tools/op_profile.py [--batch 16] [--steps 3] [--top 60]
"""
import argparse
import os
import sys
from collections import defaultdict

import torch
import torch.nn as nn

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "multimodal-deepfake-detection_amd"), REPO]

import xcp  # noqa: E402
from xcp import _lib, ddp  # noqa: E402
from Models.XceptionLSTMV import XceptionLSTMV  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=16)
    ap.add_argument("--frames", type=int, default=None)
    ap.add_argument("--model", choices=["lstmv", "lstma"], default="lstmv")
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--top", type=int, default=60)
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    xcp.set_compute_dtype("bf16")
    xcp.load_library()
    torch.manual_seed(0)
    audio = args.model == "lstma"
    args.frames = args.frames or (120 if audio else 16)
    if audio:   # bench.py --model lstma: frozen backbone, Adam 1e-4
        from Models.XceptionLSTMA import XceptionLSTMA
        model = XceptionLSTMA(512, pretrained=False)
    else:
        model = XceptionLSTMV(128, pretrained=False)
        for p in model.feature_extractor.parameters():
            p.requires_grad = True
    model = model.to(dev).train()
    params = [p for p in model.parameters() if p.requires_grad]
    buckets = ddp.GradBuckets(params, world=1)
    opt = torch.optim.Adam(params, lr=1e-5, weight_decay=1e-4, fused=True)   # one fused launch per step
    crit = nn.BCELoss()
    clips = torch.randn((args.batch, args.frames, 3, 13), device=dev) if audio else \
        torch.rand((args.batch, args.frames, 3, 299, 299), device=dev)
    labels = torch.randint(0, 2, (args.batch, 1), device=dev).float()

    def step():
        buckets.zero()
        prob = model(model.extract_features(clips, dev))
        crit(prob, labels).backward()
        buckets.allreduce()
        torch.nn.utils.clip_grad_norm_(params, 1.0)
        opt.step()

    step()
    torch.cuda.synchronize()
    rec = []
    real = _lib.call

    def timed(name, *a):
        if name in _lib.SIZE_QUERIES:
            return real(name, *a)
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        r = real(name, *a)
        e.record()
        key = (name, tuple(v for v in a if isinstance(v, int) and not isinstance(v, bool) and abs(v) < 1 << 31))
        rec.append((key, s, e))
        return r

    _lib.call = timed
    s0, e0 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s0.record()
    for _ in range(args.steps):
        step()
    e0.record()
    torch.cuda.synchronize()
    _lib.call = real
    total = s0.elapsed_time(e0) / args.steps
    agg = defaultdict(lambda: [0, 0.0])
    for key, s, e in rec:
        agg[key][0] += 1
        agg[key][1] += s.elapsed_time(e)
    rows = sorted(agg.items(), key=lambda kv: -kv[1][1])
    covered = sum(v[1] for v in agg.values()) / args.steps
    print(f"step {total:.2f} ms; xcp entry points {covered:.2f} ms per step")
    print(f"{'entry point':22s} {'calls/step':>10s} {'ms/step':>8s} {'us/call':>8s}  int args")
    for (name, ints), (n, ms) in rows[:args.top]:
        print(f"{name:22s} {n / args.steps:10.1f} {ms / args.steps:8.3f} {1e3 * ms / n:8.1f}  {ints}")


if __name__ == "__main__":
    main()
