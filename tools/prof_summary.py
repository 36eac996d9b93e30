"""Summarise a rocprofv3 kernel trace (kernel_trace CSV or SQLite .db): per-kernel total /
average time and share of GPU time, then per (kernel instance, grid) -- the shape-level view
that bench.py's live HIP-event timing is compared against.

rocprofv3 reports some dispatches of one instantiation under its mangled name and others
under a lossy demangled one ("gemm_nt_kernel<bool _Accum, int, E, 2, 2>"); dispatches are
therefore grouped on (base name, grid, workgroup, LDS, VGPRs) and labelled with the decoded
mangled name seen in that group.

With --op-order (the JSON bench.py writes under XCP_BENCH_OP_ORDER=<file>: one step's ops in call
order with their shapes and launch stream) the weight-gradient GEMM launches of every complete step
are matched to their op calls, stream by stream, and listed per shape (the middle-flow 728 x 728 one
is bench.py's roofline_wgrad op).

usage: python tools/prof_summary.py <kernel_trace.csv | .db | dir> [top] [--op-order order.json]
"""
import json
import csv
import glob
import os
import re
import sqlite3
import sys
from collections import defaultdict

_TYPES = {"DF16b": "bf16", "f": "float", "d": "double", "h": "u8", "i": "int"}


def decode(name):
    """Decode the mangled names of this repo's kernels: _ZN12_GLOBAL__N_1<n><ident>I<args>E..."""
    m = re.match(r"_ZN12_GLOBAL__N_1(\d+)(\w+)", name)
    if not m:
        return None
    n = int(m.group(1))
    ident = m.group(2)[:n]
    rest = m.group(2)[n:]
    args = []
    if rest.startswith("I"):
        body = rest[1:]
        while body and not body.startswith("EE") and not body.startswith("Ev"):
            mm = re.match(r"Li(-?\d+)E|Lb([01])E|(DF16b|f|d|h|i)", body)
            if not mm:
                break
            if mm.group(1) is not None:
                args.append(mm.group(1))
            elif mm.group(2) is not None:   # bool template argument (e.g. the NT GEMM's BN-statistics epilogue)
                args.append("true" if mm.group(2) == "1" else "false")
            else:
                args.append(_TYPES[mm.group(3)])
            body = body[mm.end():]
    return f"{ident}<{', '.join(args)}>" if args else ident


def base(name):
    m = re.search(r"(\w+_kernel)", name)
    if m:
        b = m.group(1)
        return re.sub(r"^\d+", "", b.replace("_ZN12_GLOBAL__N_1", ""))
    n = name.replace("void ", "").split("(")[0]
    return n[:60]


def load(path):
    rows = []
    if path.endswith(".db"):
        c = sqlite3.connect(path)
        for name, dur, grid, wg, lds, vgpr in c.execute(
                "select name, duration, grid_x, workgroup_x, lds_size, vgpr_count from kernels order by start"):
            rows.append((name, dur, (grid, wg, lds, vgpr)))
    else:
        with open(path) as f:
            for r in csv.DictReader(f):
                key = (r.get("Grid_Size_X"), r.get("Workgroup_Size_X"), r.get("LDS_Block_Size"), r.get("VGPR_Count"))
                rows.append((r["Kernel_Name"], int(r["End_Timestamp"]) - int(r["Start_Timestamp"]), key))
    return rows


def main():
    argv = list(sys.argv[1:])
    order = None
    if "--op-order" in argv:
        i = argv.index("--op-order")
        order = argv[i + 1]
        del argv[i:i + 2]
    path = argv[0]
    top = int(argv[1]) if len(argv) > 1 else 40
    if os.path.isdir(path):
        cands = glob.glob(os.path.join(path, "**", "*kernel_trace.csv"), recursive=True) + \
            glob.glob(os.path.join(path, "**", "*.db"), recursive=True)
        path = cands[0]
    rows = load(path)
    # instances: (base name, grid, workgroup, LDS, VGPRs) refined by the decoded template arguments
    # where rocprofv3 kept the mangled name (so e.g. gemm_nt256p_kernel<true> -- the forward, with the
    # BN-statistics epilogue -- and <false> -- the input gradient -- are separate rows)
    labels = {}
    by_base = defaultdict(lambda: [0, 0])
    by_inst = defaultdict(lambda: [0, 0])
    for name, dur, key in rows:
        b = base(name)
        by_base[b][0] += dur
        by_base[b][1] += 1
        d = decode(name)
        ik = (b,) + key + ((d,) if d and "<" in d else ())
        if d:
            labels[ik] = d
        by_inst[ik][0] += dur
        by_inst[ik][1] += 1
    total = sum(t for t, _ in by_base.values())
    print(f"source: {path}\ntotal kernel time {total / 1e6:.3f} ms over {len(rows)} dispatches\n")
    print(f"{'kernel':60s} {'calls':>6s} {'total ms':>10s} {'avg us':>9s} {'%':>6s}")
    for k, (t, c) in sorted(by_base.items(), key=lambda kv: -kv[1][0])[:top]:
        print(f"{k:60s} {c:6d} {t / 1e6:10.3f} {t / c / 1e3:9.1f} {100 * t / total:6.2f}")
    print(f"\nper instance and grid (grid = work-items, x)\n{'kernel instance':44s} {'grid':>10s} {'wg':>4s} "
          f"{'calls':>6s} {'total ms':>10s} {'avg us':>9s} {'%':>6s}")
    for k, (t, c) in sorted(by_inst.items(), key=lambda kv: -kv[1][0])[:top]:
        lab = labels.get(k, k[0])
        print(f"{lab[:44]:44s} {str(k[1]):>10s} {str(k[2]):>4s} {c:6d} {t / 1e6:10.3f} {t / c / 1e3:9.1f} "
              f"{100 * t / total:6.2f}")
    if path.endswith(".csv"):
        contention(path)
        if order:
            with open(order) as f:
                tn_by_shape(path, json.load(f))


# the roofline kernels of bench.py, (kernel base name, grid) at the bench's middle-flow shape
ROOF = (("gemm_nt256p_kernel", 131072), ("dw_fwd_w2_kernel", 1507328))


def phase_of(rows):
    """'fwd' / 'bwd' per dispatch: a step runs from one optimizer launch (opt_adam_kernel) to the
    next; its backward starts at the first kernel on a stream other than the main one (the
    weight-gradient side stream) -- dispatches of the step before that are the forward."""
    order = sorted(range(len(rows)), key=lambda i: rows[i][1])
    main = rows[order[0]][3] if rows else None
    ph, cur = [None] * len(rows), "fwd"
    for i in order:
        name = rows[i][0]
        if rows[i][3] != main and cur == "fwd":
            cur = "bwd"
        ph[i] = cur
        if "opt_adam_kernel" in name:
            cur = "fwd"
    return ph


def contention(path):
    """Launches of the roofline kernels split by step phase (forward: the pointwise GEMM with its
    BN-statistics epilogue, the op bench.py times; backward: the input-gradient GEMM) and by whether
    another stream ran a kernel during them (the side-stream weight gradients of the backward).  The
    op bench.py times live is the forward launch plus, for the pointwise GEMM, the op's second launch:
    the sparse last round on the 128x128 kernel (grid 61440 at the step shape), listed per phase too."""
    with open(path) as f:
        rows = [(r["Kernel_Name"], int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r.get("Stream_Id"),
                 int(r.get("Grid_Size_X") or 0)) for r in csv.DictReader(f)]
    ph = phase_of(rows)
    print("\nroofline kernels per step phase: launches alone on the GPU vs overlapping another stream's kernels")
    for name, grid in ROOF + (("gemm_nt_kernel", 61440),):
        for phase in ("fwd", "bwd"):
            alone, shared = [], []
            for i, r in enumerate(rows):
                if base(r[0]) != name or r[4] != grid or ph[i] != phase:
                    continue
                ov = any(o[3] != r[3] and o[1] < r[2] and o[2] > r[1] for o in rows if o is not r)
                (shared if ov else alone).append((r[2] - r[1]) / 1e3)
            if not alone and not shared:
                continue
            f = lambda v: f"{len(v):5d} x {sum(v) / len(v):7.1f} us" if v else "    0"   # noqa: E731
            print(f"{name[:22]:22s} {phase} grid {grid:>8d}  all {f(alone + shared)}  alone {f(alone)}  "
                  f"overlapped {f(shared)}")
    # the op bench.py's "roofline" times: the middle-flow 728 x 728 pointwise GEMM with its BN statistics,
    # i.e. a forward persistent launch that follows the 19^2 x 736 depthwise forward and is followed by
    # the sparse last round (grid 61440) -- the persistent kernel's grid is 256 workgroups for every
    # shape with >= 256 tiles, so the grid alone does not identify the op
    seq = sorted([r for r in rows if r[3] == rows[0][3]], key=lambda r: r[1]) if rows else []
    ops_ = []
    for i in range(1, len(seq) - 1):
        if (base(seq[i][0]) == "gemm_nt256p_kernel" and base(seq[i - 1][0]) == "dw_fwd_w2_kernel"
                and seq[i - 1][4] == 1507328 and base(seq[i + 1][0]) == "gemm_nt_kernel" and seq[i + 1][4] == 61440):
            ops_.append(((seq[i][2] - seq[i][1]) / 1e3, (seq[i + 1][2] - seq[i + 1][1]) / 1e3,
                         (seq[i + 1][2] - seq[i][1]) / 1e3))
    if ops_:
        n = len(ops_)
        m = [sum(o[k] for o in ops_) / n for k in range(3)]
        print(f"middle-flow forward op (728 x 728 @19^2 + BN statistics): {n} x persistent {m[0]:.1f} us + "
              f"sparse round {m[1]:.1f} us = {m[0] + m[1]:.1f} us of kernel time, {m[2]:.1f} us first start to "
              f"last end (bench.py's live figure: HIP events around the op)")


TN_KERNELS = ("gemm_tn256_kernel", "gemm_tn_kernel")
PEAK_BF16_TF = 2500.0


def tn_by_shape(path, order):
    """Weight-gradient GEMM launches per shape: in each step (opt_adam_kernel to opt_adam_kernel) the
    gemm_tn launches of the main stream and of the other stream(s) are matched, in start order, to the
    step's gemm_tn op calls on that stream (one launch per call); steps whose launch count differs from
    the op log's (the partial first / last step of the trace) are skipped."""
    with open(path) as f:
        rows = sorted([(r["Kernel_Name"], int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r.get("Stream_Id"))
                       for r in csv.DictReader(f)], key=lambda r: r[1])
    if not rows:
        return
    main = rows[0][3]
    want = {k: [d for d in order if d["op"] == "gemm_tn" and d["stream"] == k] for k in ("main", "side")}
    steps, cur = [], {"main": [], "side": []}
    for r in rows:
        if base(r[0]) in TN_KERNELS:
            cur["main" if r[3] == main else "side"].append(r)
        if "opt_adam_kernel" in r[0]:
            steps.append(cur)
            cur = {"main": [], "side": []}
    per = defaultdict(list)
    used = 0
    for st in steps:
        if any(len(st[k]) != len(want[k]) for k in want):
            continue
        used += 1
        for k in want:
            for d, r in zip(want[k], st[k]):
                ov = any(o[3] != r[3] and o[1] < r[2] and o[2] > r[1] for o in rows if o is not r)
                per[(k, d["M"], d["N"], d["K"], base(r[0]))].append(((r[2] - r[1]) / 1e3, ov))
    print(f"\nweight-gradient GEMM per shape ({used} complete steps; flops 2 M N K over the launch; "
          f"'shared': another stream's kernel overlapped it)")
    print(f"{'stream':6s} {'M':>9s} {'N':>5s} {'K':>5s} {'kernel':18s} {'n':>4s} {'avg us':>8s} {'alone us':>9s} "
          f"{'shared us':>9s} {'TF/s':>7s} {'frac':>6s}")
    for key, v in sorted(per.items(), key=lambda kv: -sum(x for x, _ in kv[1])):
        k, M, N, K, kern = key
        d = [x for x, _ in v]
        al = [x for x, o in v if not o]
        sh = [x for x, o in v if o]
        avg = sum(d) / len(d)
        tf = 2.0 * M * N * K / (avg * 1e-6) / 1e12
        f = lambda u: f"{sum(u) / len(u):9.1f}" if u else f"{'-':>9s}"   # noqa: E731
        print(f"{k:6s} {M:9d} {N:5d} {K:5d} {kern[:18]:18s} {len(d):4d} {avg:8.1f} {f(al)} {f(sh)} {tf:7.1f} "
              f"{tf / PEAK_BF16_TF:6.3f}")


if __name__ == "__main__":
    main()
