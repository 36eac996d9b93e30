"""Host (Python + launch) time per phase of the bench's headline step against the device time of the
same phases: is the CPU ever behind the GPU?  Runs bench.Run (XceptionLSTMV, 16 clips x 16 x 299^2,
unfrozen, bf16) eagerly; per step: host time of forward+loss / backward / all-reduce+optimizer
(time.perf_counter around the calls, no synchronisation inside the loop) and device time of the same
phases (HIP events).  Also the host time of feature_extractor.to(device) (the reference's per-step call
in extract_features).

  python tools/cpu_overhead.py      # GPU box
"""
import argparse
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "multimodal-deepfake-detection_amd"), REPO]


def main():
    import torch
    import bench
    import xcp
    from xcp import ddp
    xcp.set_compute_dtype("bf16")
    xcp.load_library()
    sys.argv = [sys.argv[0], "--mode", "unfrozen"]
    args = bench.parse()
    dev = torch.device("cuda", 0)
    run = bench.Run(args, "unfrozen", dev, 0, 1)
    for _ in range(3):
        run.step()
    torch.cuda.synchronize()
    host = {"fwd": [], "bwd": [], "opt": [], "step": []}
    evs = []
    for i in range(10):
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(4)]
        t0 = time.perf_counter()
        ev[0].record()
        run.buckets.zero()
        ddp.broadcast_buffers(run.model)
        out = run.model(run.model.extract_features(run.x, run.dev))
        loss = run.crit(out, run.y)
        ev[1].record()
        t1 = time.perf_counter()
        loss.backward()
        ev[2].record()
        t2 = time.perf_counter()
        run.buckets.allreduce()
        run.opt.step()
        ev[3].record()
        t3 = time.perf_counter()
        host["fwd"].append(t1 - t0)
        host["bwd"].append(t2 - t1)
        host["opt"].append(t3 - t2)
        host["step"].append(t3 - t0)
        evs.append(ev)
    torch.cuda.synchronize()
    dv = {"fwd": [e[0].elapsed_time(e[1]) for e in evs], "bwd": [e[1].elapsed_time(e[2]) for e in evs],
          "opt": [e[2].elapsed_time(e[3]) for e in evs], "step": [e[0].elapsed_time(e[3]) for e in evs]}
    for k in host:
        h = sorted(host[k])[len(host[k]) // 2] * 1e3
        d = sorted(dv[k])[len(dv[k]) // 2]
        print(f"{k:5s}: host {h:7.2f} ms   device {d:7.2f} ms", flush=True)
    fe = run.model.feature_extractor
    t0 = time.perf_counter()
    for _ in range(20):
        fe.to(dev)
    print(f"feature_extractor.to(device): {(time.perf_counter() - t0) / 20 * 1e3:.2f} ms host", flush=True)


if __name__ == "__main__":
    main()
