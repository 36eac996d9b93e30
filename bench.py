"""Throughput benchmark: XceptionLSTMV 16x299x299 clip training on MI355X (bf16).

BASELINE.json metric: "clips/sec (node) XceptionLSTMV 16x299x299 bf16 train at
1/2/4/8 MI355X".  One step = one training pass over b clips per GPU (synthetic,
on-device, seeded per rank): backbone (train-mode BN) -> LSTM(128) -> FC head ->
BCELoss -> backward (gradient all-reduce over RCCL overlapped with it) ->
clip_grad_norm_(1.0) -> Adam(lr 1e-5, wd 1e-4) (train_visual.py:533-577 semantics).
The headline is the unfrozen backbone (train_visual.py:551-556, every epoch after the
3rd); the frozen backbone (as shipped, XceptionLSTMV.py:15-16) is measured in the same
run and reported under "frozen".

Other configurations (secondary lines, BASELINE.json configs):
  --model xception : C2, Xception(num_classes=1) trained per frame, 64 frames of 299^2
                     (BCEWithLogits, Adam) -> frames/s
  --model lstma    : C4, XceptionLSTMA(512) on MFCC clips [b, 120, 3, 13] resized to 64^2
                     on the GPU, frozen backbone as shipped, Adam lr 1e-4 (train_audio.py:33-44)
  --model auface   : C5, the train_au_face.py step (xcp/auface.py) on the build-defined
                     AUFaceCrossDetector: 32 clips/GPU x 75 face frames of 128^2 + 17 AU crops of
                     64^2, autocast + GradScaler, accumulation 4, AdamW, OneCycleLR, averaged
                     model; a step is one micro-batch (the optimizer steps on every 4th)

Launch: ``python bench.py [--gpus N --steps K --warmup W]``.  Under torch.distributed.run
(WORLD_SIZE set) one process drives one GPU; with --gpus N > 1 and no WORLD_SIZE this
process starts N ranks itself through torch.distributed.run (before touching the GPU) and
exits with their status.  Rank 0 prints ONE JSON line.
"""
import argparse
import json
import math
import os
import subprocess
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
for _p in (os.path.join(REPO, "multimodal-deepfake-detection_amd"), REPO):
    if _p not in sys.path:
        sys.path.insert(0, _p)

PEAK_BF16_TFLOPS = 2500.0   # MI355X dense bf16 MFMA (MI355X_MICROARCH.md, spec)
PEAK_HBM_GBS = 8000.0       # MI355X HBM3E (spec)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--model", choices=["lstmv", "lstma", "xception", "auface"], default="lstmv")
    ap.add_argument("--aus", type=int, default=17, help="auface: AU crops per clip")
    ap.add_argument("--au-size", type=int, default=64, help="auface: AU crop size")
    ap.add_argument("--batch", type=int, default=None, help="clips (frames for xception) per GPU")
    ap.add_argument("--frames", type=int, default=None, help="frames per clip (default 16; 120 for lstma)")
    ap.add_argument("--size", type=int, default=299)
    ap.add_argument("--mode", choices=["unfrozen", "frozen", "both"], default=None,
                    help="backbone training (lstmv default: both, unfrozen is the headline; lstma: frozen)")
    ap.add_argument("--dtype", choices=["bf16", "fp32"], default="bf16")
    ap.add_argument("--cpu-baseline", choices=["on", "off"], default="on")
    ap.add_argument("--cpu-steps", type=int, default=3)
    ap.add_argument("--no-kernel-timing", action="store_true")
    ap.add_argument("--graph", choices=["auto", "on", "off"], default="auto",
                    help="replay the whole train step as one HIP graph (on: world size 1; auto = on for lstma only, "
                         "measured slower on the others)")
    ap.add_argument("--ddp-proxy", type=int, default=0, metavar="G",
                    help="world size 1 only: at every bucket-ready point launch a stand-in of a G-rank RCCL all-reduce "
                         "(xcp_comm_proxy) from the stream the real one would use, and report its timings "
                         "(xcp.ddp proxy mode, profiles/r06_ddp_proxy.txt); 0 = off")
    ap.add_argument("--ddp-proxy-busbw", type=float, default=300.0, help="stand-in all-reduce bus bandwidth, GB/s")
    ap.add_argument("--ddp-proxy-blocks", type=int, default=32, help="stand-in workgroups (RCCL channel blocks)")
    ap.add_argument("--small-batch", type=int, default=4,
                    help="lstmv: also time the unfrozen step at this many clips/GPU (train_visual.py:545 uses 4; "
                         "0: off)")
    ap.add_argument("--measured-peaks", choices=["on", "off"], default="on",
                    help="time a bf16 GEMM (torch.matmul -> hipBLASLt, 8192^3) and a device copy after the timed "
                         "region and report the roofline fractions against them too")
    ap.add_argument("--diag", choices=["on", "off"], default="on",
                    help="per-step / forward / backward device times, allocator counters over the timed region, "
                         "the MFMA-load clock before and after it, and (lstmv) the unfrozen step with the weight "
                         "gradients on the main stream")
    ap.add_argument("--optim", choices=["fused", "torch"], default="fused",
                    help="fused: xcp.optim.FusedAdamClip (clip + Adam in two HIP launches); torch: "
                         "clip_grad_norm_ + torch.optim.Adam(fused=True)")
    a = ap.parse_args()
    audio = a.model == "lstma"
    if a.model == "auface":
        a.frames = a.frames or 75
        a.batch = a.batch or 32
        a.size = 128 if a.size == 299 else a.size
        a.mode = a.mode or "unfrozen"
        # whole accumulation cycles (train_au_face.py: accumulation 4): the warm-up covers at least
        # one, so the first optimizer step (state allocation, the first averaged-model update) is
        # outside the timed region, and the timed window is a whole number of cycles
        acc = 4
        a.warmup = max(acc, -(-a.warmup // acc) * acc)
        a.steps = max(acc, -(-a.steps // acc) * acc)
    a.frames = a.frames or (120 if audio else 16)
    a.batch = a.batch or (64 if a.model == "xception" else 16)
    a.mode = a.mode or ("frozen" if audio else "unfrozen" if a.model == "xception" else "both")
    if audio:
        a.size = 64
    return a


def launch_ranks(args):
    """--gpus N without a torch.distributed.run parent: start N ranks (one per GPU) through it.
    Runs before any GPU call in this process; the ranks inherit stdout (rank 0 prints the line)."""
    port = 29400 + os.getpid() % 1000
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr=127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY=os.environ.get("HSA_ENABLE_IPC_MODE_LEGACY", "0"))
    return subprocess.call(cmd, env=env)


def graph_mode(args, world):
    """Replay the train step as one HIP graph (--graph on; world size 1 only: the multi-rank step
    launches RCCL collectives from inside the backward).  auto: on for the C4 line only.  The headline
    step measured 1.1 % (round 4) and 4.6 % (round 6) slower replayed than launched eagerly
    (profiles/r04_graph_ab.txt, r06_graph_ab.txt) -- the replay spreads the step's nodes over four
    hardware queues with a barrier on every cross-queue edge; the C4 step (120 per-step LSTM backward
    launches of ~8 us) +1.2 % replayed."""
    if world != 1 or args.model == "auface":
        return False
    return args.graph == "on" or (args.graph == "auto" and args.model == "lstma")


def middle_hw(size):
    """Spatial size of the 728-channel middle flow: stem conv1 s2, conv2, then three s2 blocks."""
    h = (size - 3) // 2 + 1 - 2
    for _ in range(3):
        h = (h - 1) // 2 + 1
    return h


# ------------------------------------------------------------------------------ step roofline
BLOCKS = [(64, 128, 2, 2, False, True), (128, 256, 2, 2, True, True), (256, 728, 2, 2, True, True)] + \
    [(728, 728, 3, 1, True, True)] * 8 + [(728, 1024, 2, 2, True, False)]   # Xception.py:125-140


# (cout, cin) of the units whose BN apply + pointwise dgrad + wgrad run fused in bf16
FUSED_UNITS = {(128, 64), (128, 128), (256, 128), (256, 256)}
# (cout, cin) of the units whose depthwise + pointwise forward run as one kernel in bf16 (sepfwd.hip)
SEP_FUSED_UNITS = {(128, 64), (128, 128), (256, 128)}


def step_roofline(size, frames, unfrozen, s=2):
    """Ideal time of one backbone step of this design: sum over its kernels of
    max(flops / MFMA peak, bytes / HBM peak), with each kernel's algorithmic flops and the
    bytes it must move (read its inputs once, write its outputs once; s = bytes per element).
    Returns (ms, total flops, total bytes).  The LSTM / FC head (< 0.1 % of the flops) is left
    out.  SURVEY §8(d): step roofline time = sum_ops max(flops/peak_flops, bytes/peak_bw)."""
    ops_ = []

    def op(fl, by):
        ops_.append((fl, by))

    n = frames
    oh1 = (size - 3) // 2 + 1
    oh2 = oh1 - 2
    p1, p2 = n * oh1 * oh1, n * oh2 * oh2
    op(2 * 27 * 32 * p1, 4 * 3 * n * size * size + s * 32 * p1)                  # conv1
    op(0, s * 32 * p1 * 3)                                                      # bn1 stats + apply
    op(2 * 288 * 64 * p2, s * (32 * p1 + 64 * p2))                              # conv2 (+stats)
    ps1 = n * ((oh2 - 1) // 2 + 1) ** 2
    op(0, s * 64 * ps1 * 2)           # bn2 + ReLU at block1's skip stride only (the depthwise applies it on load)
    bwd = []
    h = oh2

    def unit(cin, cout, hw, reduce=False):
        P = n * hw * hw
        if s == 2 and (cout, cin) in SEP_FUSED_UNITS:           # depthwise + pointwise in one pass
            op(2 * P * cin * cout, s * P * (2 * cin + cout) + 36 * cin)
        else:
            op(0, 2 * s * P * cin + 36 * cin)                   # depthwise fwd (BN+ReLU on load)
            op(2 * P * cin * cout, s * P * (cin + cout))        # pointwise (+BN stats epilogue)
        # BN backward: apply (read dz, y; write dy); its reduce comes fused from the consumer's
        # depthwise backward / the max-pool backward, except after a residual / the avg-pool
        if s == 2 and (cout, cin) in FUSED_UNITS:   # apply + dgrad + wgrad in one pass (unitbwd.hip)
            bwd.append((4 * P * cin * cout, s * P * (2 * cout + 2 * cin) + (2 * s * P * cout if reduce else 0)))
        else:
            bwd.append((0, (5 if reduce else 3) * s * P * cout))
            bwd.append((2 * P * cin * cout, s * P * (cin + cout)))  # pointwise dgrad
            bwd.append((2 * P * cin * cout, s * P * (cin + cout)))  # pointwise wgrad
        bwd.append((0, 3 * s * P * cin))                        # depthwise dgrad + wgrad (+BN partials)

    for cin, cout, reps, stride, _, grow in BLOCKS:
        filt = [(cin, cout)] + [(cout, cout)] * (reps - 1) if grow else [(cin, cin)] * (reps - 1) + [(cin, cout)]
        for i, (a, b) in enumerate(filt):
            unit(a, b, h, reduce=(i == len(filt) - 1 and stride == 1))
        oh = (h - 1) // stride + 1
        P, Ps = n * h * h, n * oh * oh
        if stride != 1 or cin != cout:
            op(2 * Ps * cin * cout, s * Ps * (cin + cout))                      # skip conv (+stats)
            bwd.append((0, 5 * s * Ps * cout))                                  # skip BN backward
            bwd.append((4 * Ps * cin * cout, 2 * s * Ps * (cin + cout)))        # skip dgrad + wgrad
        op(0, s * (P * cout + 2 * Ps * cout) + (Ps * cout if stride != 1 else 0))   # tail (BN, pool, add)
        if stride != 1:
            bwd.append((0, s * (Ps * cout + 2 * P * cout) + Ps * cout))        # max-pool backward (+BN reduce)
        else:
            bwd.append((0, s * P * cout))                                       # residual gradient read
        h = oh
    unit(1024, 1536, h)
    unit(1536, 2048, h, reduce=True)
    op(0, s * n * h * h * 2048)                                                 # bn4 + ReLU + avgpool
    if unfrozen:
        bwd.append((0, 2 * s * n * h * h * 2048))                               # avgpool backward
        bwd.append((0, 3 * s * 64 * p2))                   # bn2 backward apply (reduce fused: block1 depthwise)
        bwd.append((2 * 576 * 32 * p1, s * (64 * p2 + 32 * p1)))               # conv2 dgrad
        bwd.append((2 * 288 * 64 * p2, s * (64 * p2 + 32 * p1)))                # conv2 wgrad
        bwd.append((0, 5 * s * 32 * p1))                                        # bn1 backward
        bwd.append((2 * 27 * 32 * p1, 4 * 3 * n * size * size + s * 32 * p1))  # conv1 wgrad
        ops_.extend(bwd)
    ms = sum(max(fl / (PEAK_BF16_TFLOPS * 1e12), by / (PEAK_HBM_GBS * 1e9)) for fl, by in ops_) * 1e3
    return ms, sum(fl for fl, _ in ops_), sum(by for _, by in ops_)


# ------------------------------------------------------------------------------ CPU baseline
def host_cores():
    """CPUs this process may use: its affinity, capped by a cgroup CPU quota when one is set."""
    n = len(os.sched_getaffinity(0))
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            n = min(n, max(1, int(int(q) / int(per))))
    except (OSError, ValueError):
        pass
    return n


def log(msg):
    print(f"[bench {time.strftime('%H:%M:%S')}] {msg}", file=sys.stderr, flush=True)


def cpu_baseline(args, frames):
    """Oracle (oracle/xception_oracle.py: the CPU fp32 restatement of the reference, PyTorch on
    every host core this process may run on) on a bounded sample: one clip of the same shape,
    1 warm-up + cpu_steps timed full train steps (forward, BCE, backward, clip_grad_norm_, Adam),
    for each backbone mode the GPU line reports."""
    import torch
    from Models.XceptionLSTMA import XceptionLSTMA
    from Models.XceptionLSTMV import XceptionLSTMV
    from oracle import xception_oracle as O
    cores = host_cores()
    torch.set_num_threads(cores)
    torch.manual_seed(0)
    audio = args.model == "lstma"
    sd = (XceptionLSTMA(512, pretrained=False) if audio else XceptionLSTMV(128, pretrained=False)).state_dict()
    gen = torch.Generator().manual_seed(1234)
    x = torch.randn((1, frames, 3, 13), generator=gen) if audio else \
        torch.rand((1, frames, 3, args.size, args.size), generator=gen)
    y = torch.tensor([[1.0]])
    optim = dict(lr=1e-4, weight_decay=0.0, max_norm=None) if audio else dict(lr=1e-5, weight_decay=1e-4, max_norm=1.0)
    modes = ["unfrozen", "frozen"] if args.mode == "both" else [args.mode]
    res = {}
    for mode in modes:
        log(f"cpu baseline {mode}: {cores} threads, 1 + {args.cpu_steps} steps")
        O.clip_step(sd, x, y, mode == "unfrozen", audio=audio, optim=optim)
        t0 = time.perf_counter()
        for _ in range(args.cpu_steps):
            O.clip_step(sd, x, y, mode == "unfrozen", audio=audio, optim=optim)
        res[mode] = args.cpu_steps / (time.perf_counter() - t0)
        log(f"cpu baseline {mode}: {res[mode]:.4f} clips/s")
    cpu_name = ""
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                cpu_name = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    head = modes[0]
    out = {"value": round(res[head], 4), "unit": "clips/s", "cores": cores, "kind": "port",
           "sample": f"{args.cpu_steps} timed + 1 warm-up {head} train steps (BCE, backward, clip, Adam) of 1 clip x "
                     f"{frames}x{'3x13 MFCC -> 64^2' if audio else f'3x{args.size}^2'}, fp32, oracle/xception_oracle.py "
                     f"(PyTorch CPU, {cores} threads = the CPUs this process may use: affinity capped by "
                     f"the cgroup quota), {cpu_name}"}
    if "frozen" in res and head != "frozen":
        out["frozen"] = round(res["frozen"], 4)
    return out


def pmc_traffic():
    """HBM bytes per launch of the two roofline ops, from the newest committed
    ``profiles/*_optraffic.json``: separate rocprofv3 FETCH_SIZE / WRITE_SIZE passes
    (tools/pmc_traffic.py, FETCH_SIZE x2 gfx950 correction) over ``tools/kbench.py roof_ops``, which
    runs exactly the bench's two timed ops at the step's shape (the pointwise op is the persistent
    256x256 launch plus the sparse last round on the 128x128 kernel: its bytes are summed over both,
    as the live timing covers both).  Returns {kernel base: (bytes, source)} or {} when absent."""
    import glob
    files = sorted(glob.glob(os.path.join(REPO, "profiles", "*_optraffic.json")))
    if not files:
        return {}
    data = json.load(open(files[-1]))
    out = {}
    for b in ("gemm_nt", "dw_fwd"):
        cand = [v for v in data.values() if v.get("base", "").startswith(b)]
        if cand:
            n = max(v["launches"] for v in cand)
            parts = [v for v in cand if v["launches"] == n]
            out[b] = (sum(v["traffic_bytes"] for v in parts),
                      f"{os.path.relpath(files[-1], REPO)}: " + " + ".join(f"{v['kernel']} grid={v['grid']}" for v in parts)
                      + f", 2*FETCH_SIZE+WRITE_SIZE per op, mean over {n} launches (tools/kbench.py roof_ops)")
    # the weight-gradient GEMM: from the newest whole-step passes (the middle-flow launches: the grid
    # with the most launches)
    steps = sorted(glob.glob(os.path.join(REPO, "profiles", "*_step_traffic.json")))
    if steps:
        data = json.load(open(steps[-1]))
        cand = [v for v in data.values() if isinstance(v, dict) and v.get("base", "").startswith("gemm_tn256")]
        if cand:
            v = max(cand, key=lambda v: v["launches"])
            out["gemm_tn"] = (v["traffic_bytes"], f"{os.path.relpath(steps[-1], REPO)}: {v['kernel']} grid={v['grid']}, "
                                                  f"2*FETCH_SIZE+WRITE_SIZE, mean over {v['launches']} launches "
                                                  f"in the step (incl. its fp32 slab writes)")
    return out


# ------------------------------------------------------------------------------ GPU runs
class Run:
    """One model + optimiser + synthetic batch on this rank; step() is one training step."""

    def __init__(self, args, mode, dev, rank, world):
        import torch
        import torch.nn as nn
        from xcp import ddp
        self.torch = torch
        self.args, self.mode, self.world = args, mode, world
        torch.manual_seed(0)
        B, T, S = args.batch, args.frames, args.size
        self.dev = dev
        if args.model == "auface":
            from Models.AUFaceModel import AUFaceCrossDetector
            from xcp.auface import AUFaceTrainer
            self.model = AUFaceCrossDetector(num_aus=max(17, args.aus)).to(dev)
            self.trainer = AUFaceTrainer(self.model, samples_per_cls=(1000, 1000), steps_per_epoch=1 << 20)
            self.trainer.train()
            g = torch.Generator(device=dev).manual_seed(1234 + rank)
            self.batch = (torch.rand((B, 3, T, S, S), generator=g, device=dev),
                          torch.rand((B, args.aus, 3, args.au_size, args.au_size), generator=g, device=dev),
                          torch.randint(0, 2, (B,), generator=g, device=dev),
                          torch.ones(B, args.aus, device=dev), torch.rand((B, args.aus), generator=g, device=dev))
            self.i = 0
            return
        if args.model == "xception":
            from Models.Xception import xception
            model = xception(num_classes=1)
            self.crit = nn.BCEWithLogitsLoss()
        elif args.model == "lstma":
            from Models.XceptionLSTMA import XceptionLSTMA
            model = XceptionLSTMA(512, pretrained=False)
            self.crit = nn.BCELoss()
        else:
            from Models.XceptionLSTMV import XceptionLSTMV
            model = XceptionLSTMV(128, pretrained=False)
            self.crit = nn.BCELoss()
        backbone = model if args.model == "xception" else model.feature_extractor
        for p in backbone.parameters():
            p.requires_grad = mode == "unfrozen"
        if args.model == "xception":
            model.fc.weight.requires_grad = model.fc.bias.requires_grad = True
        self.model = model.to(dev).train()
        self.params = list(self.model.parameters())
        proxy = ({"world": args.ddp_proxy, "busbw": args.ddp_proxy_busbw, "blocks": args.ddp_proxy_blocks}
                 if args.ddp_proxy and world == 1 else None)
        self.buckets = ddp.GradBuckets(self.params, world=world, module=self.model, proxy=proxy)
        lr, wd = (1e-4, 0.0) if args.model == "lstma" else (1e-5, 1e-4)
        self.use_graph = graph_mode(args, world)
        self.graph = None
        if args.optim == "fused":
            from xcp.optim import FusedAdamClip
            self.opt = FusedAdamClip(self.params, lr=lr, weight_decay=wd, max_norm=1.0, capturable=self.use_graph)
        else:
            self.opt = torch.optim.Adam([p for p in self.params if p.requires_grad], lr=lr, weight_decay=wd, fused=True,
                                        capturable=self.use_graph)
        g = torch.Generator(device=dev).manual_seed(1234 + rank)
        if args.model == "lstma":
            self.x = torch.randn((B, T, 3, 13), generator=g, device=dev)
        elif args.model == "xception":
            self.x = torch.rand((B, 3, S, S), generator=g, device=dev)
        else:
            self.x = torch.rand((B, T, 3, S, S), generator=g, device=dev)
        gl = torch.Generator(device=dev).manual_seed(4321 + rank)
        self.y = torch.randint(0, 2, (B, 1), generator=gl, device=dev).float()

    def capture(self):
        """Record one train step (forward, backward with the side-stream weight gradients, clip + Adam
        with device-side step counts) as a HIP graph.  Runs after the eager warm-up, which leaves every
        persistent buffer, packed-weight table and optimiser table in place; one more eager step on a
        side stream first, as torch.cuda.graph requires."""
        import torch
        cs = torch.cuda.Stream(self.dev)
        cs.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(cs):
            self.step()
        torch.cuda.current_stream().wait_stream(cs)
        torch.cuda.synchronize()
        self.graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(self.graph):
            self.gloss = self.step()
        torch.cuda.synchronize()

    def replay(self):
        """One graph-replayed train step.  The replay updates the parameters without the Python that
        bumps their autograd versions, so they are bumped here: an eager step after replays then repacks
        its weights (engine.pack's cache is keyed on the versions)."""
        from torch.autograd.graph import increment_version
        self.graph.replay()
        increment_version(self.params)
        return self.gloss

    def step(self, ev=None):
        """One training step.  ev: 4 timing events recorded on the current stream at the step's
        phase boundaries (start, after the loss, after backward, after all-reduce + optimizer)
        -- event records only, no host synchronisation."""
        from xcp import ddp
        if ev is not None:
            ev[0].record()
        if self.args.model == "auface":
            loss, _, _ = self.trainer.micro_step(self.i, 1 << 30, self.batch)
            self.i += 1
            if ev is not None:
                for e in ev[1:]:
                    e.record()
            return loss
        self.buckets.zero()
        ddp.broadcast_buffers(self.model)
        if self.args.model == "xception":
            out = self.model(self.x)
        else:
            out = self.model(self.model.extract_features(self.x, self.dev))
        loss = self.crit(out, self.y)
        if ev is not None:
            ev[1].record()
        loss.backward()
        if ev is not None:
            ev[2].record()
        self.buckets.allreduce()
        if self.args.optim == "torch":
            self.torch.nn.utils.clip_grad_norm_([p for p in self.params if p.grad is not None], 1.0)
        self.opt.step()   # (the fused optimiser clips to norm 1.0 inside)
        if ev is not None:
            ev[3].record()
        return loss


def measured_peaks(dev):
    """Live peaks on this GPU, after the timed region (report the fraction of a
    measured GEMM peak and of a measured stream-copy peak beside the spec peaks)."""
    import torch
    a = torch.randn(8192, 8192, device=dev).to(torch.bfloat16)
    c = torch.empty_like(a)
    x = torch.empty(256 << 20, device=dev, dtype=torch.bfloat16)   # 512 MB: twice the Infinity Cache
    y = torch.empty_like(x)

    def best(fn, reps=10):
        fn()
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(reps):
            fn()
        e.record()
        torch.cuda.synchronize()
        return s.elapsed_time(e) / reps * 1e-3

    from xcp import _lib, ops
    t_mm = best(lambda: torch.matmul(a, a, out=c))
    n16 = x.numel() * 2 // 16
    t_cp = best(lambda: _lib.call("xcp_stream_copy", x.data_ptr(), y.data_ptr(), n16, ops.stream()))
    t_tc = best(lambda: y.copy_(x))
    out = {"gemm_bf16_tflops": round(2.0 * 8192 ** 3 / t_mm / 1e12, 1),
           "gemm_source": "torch.matmul (hipBLASLt) bf16 8192x8192x8192, mean of 10",
           "copy_gbs": round(2.0 * x.numel() * 2 / t_cp / 1e9, 1),
           "copy_source": "streaming copy of 512 MB, 16 B per lane, 4 loads in flight per thread (xcp_stream_copy; "
                          "read + write bytes), mean of 10",
           "torch_copy_gbs": round(2.0 * x.numel() * 2 / t_tc / 1e9, 1)}
    del a, c, x, y
    torch.cuda.empty_cache()
    return out


MEM_KEYS = ("num_alloc_retries", "num_device_alloc", "num_device_free", "num_ooms")


def mem_counters(dev):
    import torch
    st = torch.cuda.memory_stats(dev)
    return {k: int(st.get(k, 0)) for k in MEM_KEYS}


def timed(run, steps, warmup, world, timer=None, diag=None):
    """Warm-up, then exactly ``steps`` timed steps between barrier + synchronize (host clock,
    max over ranks).  diag (dict): filled with per-step / per-phase device times from events
    recorded at the step's phase boundaries, and the caching allocator's counters over the
    timed region (device allocations or retries inside it would be host-synchronising work
    the warm-up did not absorb)."""
    import torch
    import torch.distributed as dist
    from xcp import ops
    graph = getattr(run, "use_graph", False)
    for _ in range(warmup):
        run.step()
    if graph and run.graph is None:
        run.capture()
        run.replay()   # (the first replay uploads the graph)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    if timer is not None:
        if graph:
            raise ValueError("per-kernel timing needs eager steps (timed(..., graph off))")
        ops.set_kernel_timer(timer)
    evs = [[torch.cuda.Event(enable_timing=True) for _ in range(4)] for _ in range(steps)] if diag is not None else None
    m0 = mem_counters(run.dev)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    for i in range(steps):
        if graph:
            if evs is not None:
                evs[i][0].record()
            loss = run.replay()
            if evs is not None:
                evs[i][3].record()
        else:
            loss = run.step(evs[i] if evs is not None else None)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    ops.set_kernel_timer(None)
    if world > 1:
        e = torch.tensor([elapsed], device=run.dev, dtype=torch.float64)
        dist.all_reduce(e, op=dist.ReduceOp.MAX)
        elapsed = e.item()
    if diag is not None:
        m1 = mem_counters(run.dev)
        st = torch.cuda.memory_stats(run.dev)
        step_ms = [evs[i][0].elapsed_time(evs[i + 1][0]) for i in range(steps - 1)] + \
                  [evs[-1][0].elapsed_time(evs[-1][3])]
        mean = lambda v: round(sum(v) / len(v), 3)   # noqa: E731
        if graph:   # (one graph launch per step: no phase boundaries inside it)
            ph = None
        else:
            ph = [[ev[k].elapsed_time(ev[k + 1]) for ev in evs] for k in range(3)]
        diag.update({"step_ms": [round(v, 2) for v in step_ms], "graph": graph,
                     "fwd_ms": mean(ph[0]) if ph else None, "bwd_ms": mean(ph[1]) if ph else None,
                     "opt_ms": mean(ph[2]) if ph else None,
                     "alloc_in_timed_region": {k: m1[k] - m0[k] for k in MEM_KEYS},
                     "reserved_peak_gb": round(st.get("reserved_bytes.all.peak", 0) / 2 ** 30, 2),
                     "allocated_peak_gb": round(st.get("allocated_bytes.all.peak", 0) / 2 ** 30, 2)})
    return elapsed, float(loss.item())


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(args))
    import torch
    import torch.distributed as dist
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # XCP_BENCH_BACKEND=gloo (test only): ranks may share a GPU (device = local rank modulo the
    # visible devices), which exercises the whole multi-rank path on a one-GPU box; the
    # measured configuration is always RCCL ("nccl"), one GPU per rank
    backend = os.environ.get("XCP_BENCH_BACKEND", "nccl")
    if backend == "gloo":
        local = local % torch.cuda.device_count()
    if world > 1:
        torch.cuda.set_device(local)
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
    dev = torch.device("cuda", local)
    # XCP_BENCH_MAIN_PRIO=high (A/B): the whole run on a stream at the device's greatest priority, so the engine's
    # weight-gradient stream (default priority) ranks below the main stream at the workgroup dispatcher
    if os.environ.get("XCP_BENCH_MAIN_PRIO", "") == "high":
        torch.cuda.set_stream(torch.cuda.Stream(dev, priority=torch.cuda.Stream.priority_range()[1]))

    import xcp
    from xcp import engine, ops
    xcp.set_compute_dtype(args.dtype)
    xcp.load_library()
    audio, single, fusion = args.model == "lstma", args.model == "xception", args.model == "auface"
    B, T, S = args.batch, args.frames, args.size
    frames = B if single else B * T
    modes = ["unfrozen", "frozen"] if args.mode == "both" else [args.mode]

    results = {}
    diag = {"device": torch.cuda.get_device_name(dev)} if args.diag == "on" else None
    if diag is not None:
        diag["clock_mhz_idle"] = round(ops.clock_probe(dev), 1)
        diag["stream_priority_range"] = list(torch.cuda.Stream.priority_range())
    proxy_rep = None
    for mode in modes:
        if rank == 0:
            log(f"{args.model} {mode}: building model")
        run = Run(args, mode, dev, rank, world)
        timer = None
        if not args.no_kernel_timing and mode == modes[0] and not audio and not fusion:
            hm = middle_hw(S)
            cp = engine.pc(728)   # the 728-channel flow's channel pitch (736: padded rows)
            timer = ops.KernelTimer({"pw_gemm_728": lambda name, a: name == "gemm_nt" and a["M"] == frames * hm * hm
                                     and a["N"] == cp and a["K"] == cp and a["stats"] is not None,
                                     "dw_fwd_728": lambda name, a: name == "dw_fwd" and a["C"] == cp and a["H"] == hm,
                                     "tn_728": lambda name, a: name == "gemm_tn" and a["M"] == frames * hm * hm
                                     and a["N"] == 728 and a["K"] == 728})
        steps = args.steps if mode == modes[0] else max(3, args.steps // 2)
        order_path = os.environ.get("XCP_BENCH_OP_ORDER")
        if order_path and mode == modes[0]:
            # one extra eager step (an additional warm-up step) whose ops are logged in call order with their
            # launch stream, for tools/prof_summary.py --op-order (shapes of a rocprofv3 trace's launches)
            oplog = []
            prev_graph, run.use_graph = run.use_graph, False
            ops.set_op_log(oplog)
            try:
                run.step()
            finally:
                ops.set_op_log(None)
                run.use_graph = prev_graph
            torch.cuda.synchronize()
            if rank == 0:
                main_stream = torch.cuda.current_stream().cuda_stream
                with open(order_path, "w") as f:
                    json.dump([dict(d, stream="main" if d["stream"] == main_stream else "side") for d in oplog], f)
        dg = {} if diag is not None else None
        if os.environ.get("XCP_BENCH_STREAM") == "high":   # A/B: the step on a high-priority stream
            hs = torch.cuda.Stream(dev, priority=torch.cuda.Stream.priority_range()[1])
            hs.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(hs):
                elapsed, loss = timed(run, steps, args.warmup, world, timer, dg)
            torch.cuda.current_stream().wait_stream(hs)
        else:
            elapsed, loss = timed(run, steps, args.warmup, world, None, dg)
        if mode == modes[0] and getattr(getattr(run, "buckets", None), "proxy", None) is not None:
            from xcp import ddp as _ddp
            proxy_rep = _ddp.proxy_report(run.buckets, steps)
        if timer is not None:
            # per-kernel durations for the roofline lines, on a second timed region of the same steps right
            # after the headline one: the bracketing HIP events cost the step 1.1-1.5 % (409.1 vs 414.5
            # clips/s, profiles/r04_kernel_timer_ab.txt), so the headline region runs without them (and a
            # graph-replayed step has no launches to bracket)
            prev_graph = run.use_graph
            run.use_graph = False
            try:
                timed(run, steps, 1, world, timer)
            finally:
                run.use_graph = prev_graph
            timer.separate = True
        if dg is not None:
            if mode == modes[0]:
                dg["clock_mhz_after"] = round(ops.clock_probe(dev), 1)
            diag[mode] = dg
        results[mode] = (elapsed, steps, loss, timer)
        if rank == 0:
            log(f"{args.model} {mode}: {1e3 * elapsed / steps:.2f} ms/step")
        if diag is not None and mode == "unfrozen" and args.model == "lstmv" and not fusion:
            # the same step with the weight gradients on the main stream (no side-stream overlap)
            prev_side, prev_graph = engine.WGRAD_SIDE_STREAM, run.use_graph
            engine.WGRAD_SIDE_STREAM = False
            run.use_graph = False   # (eager: the captured graph holds the side-stream form)
            try:
                s2 = max(3, args.steps // 2)
                e2, _ = timed(run, s2, 2, world)
                diag["unfrozen"]["wgrad_main_stream_ms"] = round(1e3 * e2 / s2, 3)
                log(f"{args.model} {mode}, weight gradients on the main stream: {1e3 * e2 / s2:.2f} ms/step")
            finally:
                engine.WGRAD_SIDE_STREAM, run.use_graph = prev_side, prev_graph
        del run
        torch.cuda.empty_cache()
    small = None
    if args.model == "lstmv" and args.small_batch and args.small_batch != B:
        # the script's own batch (train_visual.py:545), unfrozen, on every rank (the step all-reduces)
        import copy
        a4 = copy.copy(args)
        a4.batch = args.small_batch
        run = Run(a4, "unfrozen", dev, rank, world)
        s4 = max(5, args.steps // 2)
        e4, l4 = timed(run, s4, max(2, args.warmup), world)
        small = {"batch": a4.batch, "value": round(a4.batch * world * s4 / e4, 3), "ms_per_step": round(1e3 * e4 / s4, 3),
                 "steps": s4, "loss": round(l4, 5), "mode": "unfrozen"}
        del run
        torch.cuda.empty_cache()

    if rank == 0:
        head = modes[0]
        elapsed, steps, loss, timer = results[head]
        units = B * world * steps
        value = units / elapsed
        hm = middle_hw(S)
        M = frames * hm * hm
        roof, extra = None, {}
        traffic = {} if (audio or single or fusion) else pmc_traffic()   # the committed PMC passes are of the headline ops
        if timer is not None:
            pw_ms, dw_ms = timer.mean_ms("pw_gemm_728"), timer.mean_ms("dw_fwd_728")
            if pw_ms:
                flops = 2.0 * M * 728 * 728
                ach = flops / (pw_ms * 1e-3) / 1e12
                roof = {"bound": "mfma", "achieved": round(ach, 1), "peak": PEAK_BF16_TFLOPS, "unit": "TFLOP/s",
                        "frac": round(ach / PEAK_BF16_TFLOPS, 4),
                        "traffic": traffic.get("gemm_nt", (None,))[0],
                        "traffic_source": traffic.get("gemm_nt", (None, None))[1],
                        "kernel": f"gemm_nt256p_kernel + sparse last round on gemm_nt_kernel (the xcp_gemm_nt op: "
                                  f"bf16 pointwise 1x1 728->728 @{hm}x{hm} with the BN-statistics epilogue, middle flow; "
                                  f"channel pitch {engine.pc(728)}, flops counted for the 728 real channels)",
                        "flops_per_launch": flops, "avg_launch_ms": round(pw_ms, 4), "launches": timer.count("pw_gemm_728")}
            if dw_ms:
                byts = 2.0 * (2 * M * 728) + 4 * 9 * 728
                gbs = byts / (dw_ms * 1e-3) / 1e9
                extra["roofline_dw"] = {"bound": "hbm", "achieved": round(gbs, 1), "peak": PEAK_HBM_GBS, "unit": "GB/s",
                                        "frac": round(gbs / PEAK_HBM_GBS, 4),
                                        "traffic": traffic.get("dw_fwd", (None,))[0],
                                        "traffic_source": traffic.get("dw_fwd", (None, None))[1],
                                        "kernel": f"dw_fwd_w2_kernel (depthwise 3x3 C=728 @{hm}x{hm}; channel pitch "
                                                  f"{engine.pc(728)}, bytes counted for the 728 real channels)",
                                        "bytes_per_launch": byts, "avg_launch_ms": round(dw_ms, 4)}
            tn_ms = timer.mean_ms("tn_728")
            if tn_ms:   # the weight-gradient GEMM (side stream, the largest kernel by time): in-step, contended
                flops = 2.0 * M * 728 * 728
                ach = flops / (tn_ms * 1e-3) / 1e12
                extra["roofline_wgrad"] = {
                    "bound": "mfma", "achieved": round(ach, 1), "peak": PEAK_BF16_TFLOPS, "unit": "TFLOP/s",
                    "frac": round(ach / PEAK_BF16_TFLOPS, 4), "traffic": traffic.get("gemm_tn", (None,))[0],
                    "traffic_source": traffic.get("gemm_tn", (None, None))[1],
                    "kernel": f"{'gemm_tn256_kernel' if os.environ.get('XCP_TN_LOOP') == '1' else 'gemm_tn256q_kernel'} "
                              f"(split-K weight gradient dW = dY^T X of the 728->728 pointwise @{hm}x{hm}, "
                              f"side stream beside the backward's main stream; slab reduction not included)",
                    "flops_per_launch": flops, "avg_launch_ms": round(tn_ms, 4), "launches": timer.count("tn_728")}
        if timer is not None and getattr(timer, "separate", False):
            note = ("HIP events on the launch stream around every launch of the op, over a second timed region of "
                    f"{steps} eager steps of the same train step run right after the headline region (the events "
                    "cost the step 1.1-1.5 %, so the headline region runs without them)")
            for r in [roof, extra.get("roofline_dw"), extra.get("roofline_wgrad")]:
                if r:
                    r["timing"] = note
        if not audio and not fusion and args.dtype == "bf16":
            ideal, fl, by = step_roofline(S, frames, head == "unfrozen")
            ms = 1e3 * elapsed / steps
            extra["step_roofline"] = {"ideal_ms": round(ideal, 3), "ms_per_step": round(ms, 3),
                                      "frac": round(ideal / ms, 4), "flops": fl, "bytes": by,
                                      "model": "sum over the backbone's kernels of max(flops / 2.5 PF bf16, bytes / "
                                               "8 TB/s), bytes = each kernel's inputs read once + outputs written once "
                                               "(bench.py step_roofline)"}
        if "frozen" in results and head != "frozen":
            e2, s2, l2, _ = results["frozen"]
            fz = {"value": round(B * world * s2 / e2, 3), "ms_per_step": round(1e3 * e2 / s2, 3), "steps": s2,
                  "loss": round(l2, 5)}
            if not audio:
                ideal, _, _ = step_roofline(S, frames, False)
                fz["step_roofline_frac"] = round(ideal / (1e3 * e2 / s2), 4)
            extra["frozen"] = fz
        if fusion:
            metric = (f"clips/sec (node) AU+face fusion (build-defined AUFaceCrossDetector) {T}x{S}x{S} + "
                      f"{args.aus} AU x {args.au_size}x{args.au_size} {args.dtype} train")
            name, shape = "AUFaceCrossDetector(17, 512, 512, 256)", (f"{T} frames x 3x{S}x{S} + {args.aus} AU crops x "
                                                                     f"3x{args.au_size}x{args.au_size}")
        elif audio:
            metric = f"clips/sec (node) XceptionLSTMA MFCC {T}x3x13 (64x64) {args.dtype} train"
            name, shape = "XceptionLSTMA(hidden=512)", f"{T} MFCC frames x 3x13 -> 64x64"
        elif single:
            metric = f"frames/sec (node) Xception single-frame {S}x{S} {args.dtype} train"
            name, shape = "Xception(num_classes=1)", f"3x{S}x{S} frames"
        else:
            metric = "clips/sec (node) XceptionLSTMV 16x299x299 bf16 train"
            name, shape = "XceptionLSTMV(hidden=128)", f"{T} frames x 3x{S}x{S}"
        unit = "frames/s" if single else "clips/s"
        out = {"metric": metric, "value": round(value, 3), "unit": unit, "n_gpus": world, "steps": steps,
               "warmup": args.warmup, "ms_per_step": round(1e3 * elapsed / steps, 3), "higher_is_better": True,
               "scaling": "weak", "vs_baseline": None, "dtype": args.dtype,
               "data": f"synthetic (on-device {'N(0,1) MFCC' if audio else 'U[0,1)'} inputs, seeded per rank; "
                       "random-init weights, Xception.py:154-160 scheme)",
               "config": {"workload": f"{name} {head}-backbone train step, {B} {'frames' if single else 'clips'}/GPU x "
                                      f"{shape}" + ("" if fusion else f", {'BCEWithLogits' if single else 'BCE'} + "
                                                                      "clip 1.0 + Adam"),
                          "global_batch": B * world, "frames": 1 if single else T, "size": S, "mode": head,
                          "optimizer": ("CB-focal(ArcFace) + align + temporal losses, autocast + GradScaler, "
                                        "accumulation 4, clip 1.0, AdamW, OneCycleLR, averaged model (train_au_face.py)"
                                        if fusion else "clip 1.0 + Adam, " + ("xcp FusedAdamClip" if args.optim == "fused"
                                                                              else "torch fused Adam")),
                          "parallelism": f"dp{world}",
                          "execution": "one HIP graph per train step (captured after the eager warm-up, replayed)"
                          if graph_mode(args, world) else "eager launches"},
               "roofline": roof, "loss": round(loss, 5)}
        out.update(extra)
        if proxy_rep is not None:
            out["ddp_proxy"] = proxy_rep
        if small is not None:
            out["small_batch"] = small
        if diag is not None:
            out["diag"] = diag
        if args.measured_peaks == "on" and not audio and not fusion:
            mp = measured_peaks(dev)
            out["measured_peaks"] = mp
            if out.get("roofline"):
                out["roofline"]["frac_of_measured_peak"] = round(out["roofline"]["achieved"] / mp["gemm_bf16_tflops"], 4)
            if out.get("roofline_dw"):
                out["roofline_dw"]["frac_of_measured_peak"] = round(out["roofline_dw"]["achieved"] / mp["copy_gbs"], 4)
        if args.cpu_baseline == "on" and world == 1 and not single and not fusion:
            out["cpu_baseline"] = cpu_baseline(args, T)
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
