"""Is the headline step launch-bound?  Host time to ISSUE each train step (no synchronisation inside the
loop) against the device time per step: if issuing a step takes about as long as running it, the GPU
waits on the host at some point of every step.

usage: python tools/cpu_launch_probe.py [steps]
"""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "multimodal-deepfake-detection_amd"), REPO]


def main():
    import torch
    import bench
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 10
    sys.argv = [sys.argv[0], "--cpu-baseline", "off", "--mode", "unfrozen"]
    args = bench.parse()
    args.mode = args.mode or "unfrozen"
    dev = torch.device("cuda:0")
    run = bench.Run(args, args.mode, dev, 0, 1)
    for _ in range(3):
        run.step()
    torch.cuda.synchronize()
    issue = []
    t0 = time.perf_counter()
    for _ in range(steps):
        a = time.perf_counter()
        run.step()
        issue.append(time.perf_counter() - a)
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print(f"issue per step (ms): {[round(v * 1e3, 2) for v in issue]}")
    print(f"host issue total {(t1 - t0) * 1e3:.1f} ms for {steps} steps; wall incl. drain {(t2 - t0) * 1e3:.1f} ms "
          f"({(t2 - t0) * 1e3 / steps:.2f} ms/step)")
    # issue alone with the queue drained before each step (the host's own cost of one step)
    solo = []
    for _ in range(3):
        torch.cuda.synchronize()
        a = time.perf_counter()
        run.step()
        solo.append(time.perf_counter() - a)
    torch.cuda.synchronize()
    print(f"issue of one step from an idle queue (ms): {[round(v * 1e3, 2) for v in solo]}")


if __name__ == "__main__":
    main()
