"""Host-side time of the headline train step: where the Python launches spend their time, and how far
ahead of the GPU the host runs at the forward -> backward boundary (where the round-5 trace showed
~0.5 ms of main-stream idle before the backbone backward's first launch).

For a few steps after the warm-up: host timestamps at the step's phase points and at the backbone
backward's entry / its first launch (engine.pack_bwd), each paired with an event on the current stream
so that the GPU's position at that moment can be compared (host ahead = GPU work still queued); then a
cProfile of three steps (top functions by own time).

usage (GPU box): python tools/host_timeline.py [steps]
"""
import cProfile
import os
import pstats
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "multimodal-deepfake-detection_amd"), REPO]


def main():
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 4
    sys.argv = [sys.argv[0]]
    import torch
    import bench
    import xcp
    from xcp import engine
    args = bench.parse()
    dev = torch.device("cuda:0")
    xcp.set_compute_dtype("bf16")
    xcp.load_library()
    run = bench.Run(args, "unfrozen", dev, 0, 1)
    for _ in range(3):
        run.step()
    torch.cuda.synchronize()

    marks = []

    def mark(name):
        ev = torch.cuda.Event(enable_timing=True)
        ev.record()
        marks.append((name, time.perf_counter(), ev))

    real_bwd, real_pack = engine.XceptionEngine._backward, engine.XceptionEngine.pack_bwd

    def bwd(self, *a, **k):
        mark("engine._backward entry")
        return real_bwd(self, *a, **k)

    def pack(self, *a, **k):
        r = real_pack(self, *a, **k)
        mark("pack_bwd launched")
        return r

    engine.XceptionEngine._backward, engine.XceptionEngine.pack_bwd = bwd, pack
    crit_real = run.crit

    def crit(out, y):
        mark("forward enqueued")
        return crit_real(out, y)

    run.crit = crit
    real_step = run.opt.step

    def opt_step(*a, **k):
        mark("backward enqueued")
        r = real_step(*a, **k)
        mark("optimizer enqueued")
        return r

    run.opt.step = opt_step
    for _ in range(steps):
        mark("step start")
        run.step()
    torch.cuda.synchronize()
    t0h, e0 = marks[0][1], marks[0][2]
    print("host ms | GPU ms at that event (the GPU position when it is reached) | GPU lag = gpu - host")
    for name, th, ev in marks:
        tg = e0.elapsed_time(ev)
        print(f"{1e3 * (th - t0h):9.2f} {tg:9.2f} {tg - 1e3 * (th - t0h):8.2f}  {name}")
    engine.XceptionEngine._backward, engine.XceptionEngine.pack_bwd = real_bwd, real_pack
    run.crit, run.opt.step = crit_real, real_step

    # host time per step alone (no sync): how much of the GPU step the host needs
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(steps):
        run.step()
    th = time.perf_counter() - t
    torch.cuda.synchronize()
    tg = time.perf_counter() - t
    print(f"host enqueue {1e3 * th / steps:.2f} ms/step, GPU-complete {1e3 * tg / steps:.2f} ms/step")

    pr = cProfile.Profile()
    pr.enable()
    for _ in range(3):
        run.step()
    torch.cuda.synchronize()
    pr.disable()
    st = pstats.Stats(pr)
    st.sort_stats("tottime").print_stats(30)
    st.sort_stats("cumulative").print_stats(40)


if __name__ == "__main__":
    main()
