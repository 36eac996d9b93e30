"""Where the headline step's small ATen kernels come from: the ATen fill / copy / add ops of a few
steps, grouped by their Python call site (torch.profiler with stacks).

usage (GPU box): python tools/aten_sources.py [steps]
"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "multimodal-deepfake-detection_amd"), REPO]


def main():
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    sys.argv = [sys.argv[0]]
    import torch
    from torch.profiler import ProfilerActivity, profile
    import bench
    import xcp
    args = bench.parse()
    dev = torch.device("cuda:0")
    xcp.set_compute_dtype("bf16")
    xcp.load_library()
    run = bench.Run(args, "unfrozen", dev, 0, 1)
    for _ in range(3):
        run.step()
    torch.cuda.synchronize()
    with profile(activities=[ProfilerActivity.CPU], with_stack=True) as prof:
        for _ in range(steps):
            run.step()
        torch.cuda.synchronize()
    ka = prof.key_averages(group_by_stack_n=6)
    rows = [e for e in ka if e.key in ("aten::fill_", "aten::zero_", "aten::copy_", "aten::add_", "aten::zeros",
                                        "aten::zeros_like", "aten::clone", "aten::add")]
    rows.sort(key=lambda e: -e.count)
    for e in rows[:40]:
        print(f"{e.count / steps:6.1f}/step  {e.key}")
        for fr in (e.stack or [])[:6]:
            print("        ", fr)


if __name__ == "__main__":
    main()
