"""Throughput benchmark: XceptionLSTMV 16x299x299 clip training on MI355X (bf16).

BASELINE.json metric: "clips/sec (node) XceptionLSTMV 16x299x299 bf16 train at
1/2/4/8 MI355X".  One step = one training pass over b clips per GPU (synthetic,
on-device, seeded per rank): backbone (train-mode BN) -> LSTM(128) -> FC head ->
BCELoss -> backward -> gradient all-reduce (RCCL) -> clip_grad_norm_(1.0) ->
Adam(lr 1e-5, wd 1e-4) (train_visual.py:540-577 semantics).  Default mode is the
unfrozen backbone (train_visual.py:551-556, every epoch after the 3rd); the
frozen backbone (as shipped, XceptionLSTMV.py:15-16) is ``--mode frozen``.

``--model lstma`` runs the audio configuration instead (C4: XceptionLSTMA(512) on MFCC
clips [b, 120, 3, 13] resized to 64x64 on the GPU, frozen backbone as shipped,
Adam lr 1e-4, train_audio.py:33-44); it is a secondary line, not the headline metric.

Launch: ``python bench.py [--gpus N --steps K --warmup W]``; N>1 under
``torch.distributed.run`` (one rank per GPU, RANK/LOCAL_RANK/WORLD_SIZE from env).
Rank 0 prints ONE JSON line.
"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
for _p in (os.path.join(REPO, "multimodal-deepfake-detection_amd"), REPO):
    if _p not in sys.path:
        sys.path.insert(0, _p)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402
import torch.nn as nn  # noqa: E402

PEAK_BF16_TFLOPS = 2500.0   # MI355X dense bf16 MFMA (MI355X_MICROARCH.md, spec)
PEAK_HBM_GBS = 8000.0       # MI355X HBM3E (spec)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--model", choices=["lstmv", "lstma"], default="lstmv")
    ap.add_argument("--batch", type=int, default=16, help="clips per GPU")
    ap.add_argument("--frames", type=int, default=None, help="frames per clip (default 16; 120 for lstma)")
    ap.add_argument("--size", type=int, default=299)
    ap.add_argument("--mode", choices=["unfrozen", "frozen"], default=None,
                    help="backbone training (default unfrozen; frozen for lstma, as shipped)")
    ap.add_argument("--dtype", choices=["bf16", "fp32"], default="bf16")
    ap.add_argument("--cpu-baseline", choices=["on", "off"], default="on")
    ap.add_argument("--cpu-steps", type=int, default=2)
    ap.add_argument("--no-kernel-timing", action="store_true")
    ap.add_argument("--optim", choices=["fused", "torch"], default="fused",
                    help="fused: xcp.optim.FusedAdamClip (clip + Adam in two HIP launches); torch: "
                         "clip_grad_norm_ + torch.optim.Adam(fused=True)")
    a = ap.parse_args()
    audio = a.model == "lstma"
    a.frames = a.frames or (120 if audio else 16)
    a.mode = a.mode or ("frozen" if audio else "unfrozen")
    if audio:
        a.size = 64
    return a


def middle_hw(size):
    """Spatial size of the 728-channel middle flow: stem conv1 s2, conv2, then three s2 blocks."""
    h = (size - 3) // 2 + 1 - 2
    for _ in range(3):
        h = (h - 1) // 2 + 1
    return h


def cpu_baseline(args, frames):
    """Oracle (CPU fp32 restatement of the reference, oracle/) on a bounded sample:
    one clip of the same shape, 1 warm-up + cpu_steps timed train steps."""
    from Models.XceptionLSTMA import XceptionLSTMA
    from Models.XceptionLSTMV import XceptionLSTMV
    from oracle import xception_oracle as O
    cores = len(os.sched_getaffinity(0))
    cores = min(cores, int(os.environ.get("OMP_NUM_THREADS", cores)))
    torch.set_num_threads(cores)
    torch.manual_seed(0)
    audio = args.model == "lstma"
    sd = (XceptionLSTMA(512, pretrained=False) if audio else XceptionLSTMV(128, pretrained=False)).state_dict()
    gen = torch.Generator().manual_seed(1234)
    x = torch.randn((1, frames, 3, 13), generator=gen) if audio else \
        torch.rand((1, frames, 3, args.size, args.size), generator=gen)
    y = torch.tensor([[1.0]])
    unfrozen = args.mode == "unfrozen"
    O.clip_step(sd, x, y, unfrozen, audio=audio)
    t0 = time.perf_counter()
    for _ in range(args.cpu_steps):
        O.clip_step(sd, x, y, unfrozen, audio=audio)
    dt = (time.perf_counter() - t0) / args.cpu_steps
    cpu_name = ""
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                cpu_name = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    return {"value": round(1.0 / dt, 4), "unit": "clips/s", "cores": cores, "kind": "port",
            "sample": f"{args.cpu_steps} timed + 1 warm-up {args.mode} train steps of 1 clip x "
                      f"{frames}x{'3x13 MFCC -> 64^2' if audio else f'3x{args.size}^2'}, "
                      f"fp32, oracle/xception_oracle.py (PyTorch CPU), {cpu_name}"}


def pmc_traffic():
    """HBM bytes per launch of the two roofline kernels, from the newest committed
    ``profiles/*_traffic.json`` (tools/pmc_traffic.py over separate FETCH_SIZE / WRITE_SIZE
    rocprofv3 passes of this bench, FETCH_SIZE x2 gfx950 correction).  The middle-flow
    shape is the most frequent dispatch of each kernel, so it is the group with most launches.
    Returns ({kernel base: (bytes, source)}) or {} when no file exists."""
    import glob
    files = sorted(glob.glob(os.path.join(REPO, "profiles", "*_traffic.json")))
    if not files:
        return {}
    data = json.load(open(files[-1]))
    out = {}
    for b in ("gemm_nt", "dw_fwd_kernel"):
        cand = [v for v in data.values() if v.get("base", "").startswith(b)]
        if cand:
            v = max(cand, key=lambda v: v["launches"])
            out[b] = (v["traffic_bytes"], f"{os.path.relpath(files[-1], REPO)}: {v['kernel']} grid={v['grid']}, "
                                          f"2*FETCH_SIZE+WRITE_SIZE mean over {v['launches']} launches")
    return out


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    dev = torch.device("cuda", local)

    import xcp
    from xcp import ddp, ops
    from Models.XceptionLSTMA import XceptionLSTMA
    from Models.XceptionLSTMV import XceptionLSTMV
    xcp.set_compute_dtype(args.dtype)
    xcp.load_library()
    audio = args.model == "lstma"

    torch.manual_seed(0)
    model = XceptionLSTMA(512, pretrained=False) if audio else XceptionLSTMV(128, pretrained=False)
    if args.mode == "unfrozen":
        for p in model.feature_extractor.parameters():
            p.requires_grad = True
    model = model.to(dev).train()
    params = [p for p in model.parameters() if p.requires_grad]
    buckets = ddp.GradBuckets(params, world=world)
    lr, wd = (1e-4, 0.0) if audio else (1e-5, 1e-4)   # train_audio.py:33-44 / train_visual.py:540-577
    if args.optim == "fused":
        from xcp.optim import FusedAdamClip
        opt = FusedAdamClip(params, lr=lr, weight_decay=wd, max_norm=1.0)
    else:
        opt = torch.optim.Adam(params, lr=lr, weight_decay=wd, fused=True)
    crit = nn.BCELoss()

    B, T, S = args.batch, args.frames, args.size
    g = torch.Generator(device=dev).manual_seed(1234 + rank)
    clips = torch.randn((B, T, 3, 13), generator=g, device=dev) if audio else \
        torch.rand((B, T, 3, S, S), generator=g, device=dev)
    gl = torch.Generator(device=dev).manual_seed(4321 + rank)
    labels = torch.randint(0, 2, (B, 1), generator=gl, device=dev).float()

    def step():
        buckets.zero()
        ddp.broadcast_buffers(model)
        feats = model.extract_features(clips, dev)
        prob = model(feats)
        loss = crit(prob, labels)
        loss.backward()
        buckets.allreduce()
        if args.optim == "torch":
            torch.nn.utils.clip_grad_norm_(params, 1.0)
        opt.step()   # (the fused optimizer clips to norm 1.0 inside)
        return loss

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()

    timer = None
    if not args.no_kernel_timing:
        hm = middle_hw(S)
        timer = ops.KernelTimer({"pw_gemm_728": lambda name, a: name == "gemm_nt" and a["M"] == B * T * hm * hm
                                 and a["N"] == 728 and a["K"] == 728 and a["stats"] is not None,
                                 "dw_fwd_728": lambda name, a: name == "dw_fwd" and a["C"] == 728 and a["H"] == hm})
        ops.set_kernel_timer(timer)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        loss = step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    ops.set_kernel_timer(None)
    if world > 1:
        e = torch.tensor([elapsed], device=dev, dtype=torch.float64)
        dist.all_reduce(e, op=dist.ReduceOp.MAX)
        elapsed = e.item()

    clips_total = B * world * args.steps
    value = clips_total / elapsed
    out = None
    if rank == 0:
        hm = middle_hw(S)
        M = B * T * hm * hm
        roof = None
        extra = {}
        traffic = {} if audio else pmc_traffic()   # the committed PMC passes are of the headline (lstmv) bench
        if timer is not None:
            pw_ms = timer.mean_ms("pw_gemm_728")
            dw_ms = timer.mean_ms("dw_fwd_728")
            if pw_ms:
                flops = 2.0 * M * 728 * 728
                ach = flops / (pw_ms * 1e-3) / 1e12
                roof = {"bound": "mfma", "achieved": round(ach, 1), "peak": PEAK_BF16_TFLOPS, "unit": "TFLOP/s",
                        "frac": round(ach / PEAK_BF16_TFLOPS, 4),
                        "traffic": traffic.get("gemm_nt", (None,))[0],
                        "traffic_source": traffic.get("gemm_nt", (None, None))[1],
                        "kernel": f"gemm_nt256k64_kernel (bf16 pointwise 1x1 728->728 @{hm}x{hm}, middle flow)",
                        "flops_per_launch": flops, "avg_launch_ms": round(pw_ms, 4),
                        "launches": timer.count("pw_gemm_728")}
            if dw_ms:
                byts = 2.0 * (2 * M * 728) + 4 * 9 * 728
                gbs = byts / (dw_ms * 1e-3) / 1e9
                extra["roofline_dw"] = {"bound": "hbm", "achieved": round(gbs, 1), "peak": PEAK_HBM_GBS, "unit": "GB/s",
                                        "frac": round(gbs / PEAK_HBM_GBS, 4),
                                        "traffic": traffic.get("dw_fwd_kernel", (None,))[0],
                                        "traffic_source": traffic.get("dw_fwd_kernel", (None, None))[1],
                                        "kernel": f"dw_fwd_kernel<bf16> (depthwise 3x3 C=728 @{hm}x{hm})",
                                        "bytes_per_launch": byts, "avg_launch_ms": round(dw_ms, 4)}
        metric = (f"clips/sec (node) XceptionLSTMA MFCC {T}x3x13 (64x64) {args.dtype} train" if audio else
                  "clips/sec (node) XceptionLSTMV 16x299x299 bf16 train")
        name = "XceptionLSTMA(hidden=512)" if audio else "XceptionLSTMV(hidden=128)"
        shape = f"{T} MFCC frames x 3x13 -> 64x64" if audio else f"{T} frames x 3x{S}x{S}"
        out = {"metric": metric,
               "value": round(value, 3), "unit": "clips/s", "n_gpus": world, "steps": args.steps,
               "warmup": args.warmup, "ms_per_step": round(1e3 * elapsed / args.steps, 3), "higher_is_better": True,
               "scaling": "weak", "vs_baseline": None, "dtype": args.dtype, "data": f"synthetic (on-device {'N(0,1) MFCC' if audio else 'U[0,1)'} "
               "clips, seeded per rank; random-init weights, Xception.py:154-160 scheme)",
               "config": {"workload": f"{name} {args.mode}-backbone train step, {B} clips/GPU x {shape}, BCE + Adam",
                          "global_batch": B * world, "frames": T, "size": S, "mode": args.mode,
                          "optimizer": "clip 1.0 + Adam, " + ("xcp FusedAdamClip" if args.optim == "fused"
                                                               else "torch fused Adam"),
                          "parallelism": f"dp{world}"},
               "roofline": roof, "loss": round(float(loss.item()), 5)}
        out.update(extra)
    if rank == 0 and args.cpu_baseline == "on" and world == 1:
        out["cpu_baseline"] = cpu_baseline(args, T)
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
