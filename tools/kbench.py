"""Kernel micro-benchmarks at the bench's middle-flow shapes (N = 256 frames of 19x19x728,
bf16) and a few others: average launch time with HIP events, achieved GB/s or TFLOP/s.
``cold`` flushes the Infinity Cache / L2 before every launch.

usage: python tools/kbench.py [names...]   (default: copy dw_fwd dw_bwd gemm bn tail)
"""
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "multimodal-deepfake-detection_amd"), REPO]

from xcp import ops  # noqa: E402


def timeit(fn, iters=20, warm=3):
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters


def main():
    dev = torch.device("cuda:0")
    ops._lib.load()
    sel = set(sys.argv[1:]) or {"copy", "dw_fwd", "dw_bwd", "gemm", "bn", "tail"}
    dt = torch.bfloat16
    N, H, W, C = 256, 19, 19, 728
    M = N * H * W
    g = torch.Generator(device=dev).manual_seed(0)
    X = torch.randn(M, C, device=dev, generator=g).to(dt)
    Y = torch.empty_like(X)
    D = torch.randn(M, C, device=dev, generator=g).to(dt)
    Wt = torch.randn(9, C, device=dev, generator=g)
    sc = torch.rand(C, device=dev, generator=g) + 0.5
    sh = torch.randn(C, device=dev, generator=g)
    Wp = (torch.randn(C, C, device=dev, generator=g) / 27).to(dt)
    dW = torch.empty(C * 9, device=dev)
    st = {"mean": torch.zeros(C, device=dev), "invstd": torch.ones(C, device=dev)}
    tensor_bytes = M * C * 2

    def rep(name, ms, byts=None, flops=None):
        line = f"{name:40s} {ms * 1e3:9.1f} us"
        if byts:
            line += f"  {byts / ms / 1e6:8.1f} GB/s"
        if flops:
            line += f"  {flops / ms / 1e9:8.1f} TFLOP/s"
        print(line, flush=True)

    if "copy" in sel:
        rep("torch copy (ref BW)", timeit(lambda: Y.copy_(X)), 2 * tensor_bytes)
    if "dw_fwd" in sel:
        for act in (1, 2):
            rep(f"dw_fwd act={act}", timeit(lambda: ops.dw_fwd(act, X, Y, Wt, sc, sh, N, H, W, C)), 2 * tensor_bytes)
    if "dw_bwd" in sel:
        rep("dw_bwd act=2 +bnsums", timeit(lambda: ops.dw_bwd(2, D, X, Wt, sc, sh, Y, dW, N, H, W, C, bn_stats=st)),
            3 * tensor_bytes)
        rep("dw_bwd act=1 +res", timeit(lambda: ops.dw_bwd(1, D, X, Wt, sc, sh, Y, dW, N, H, W, C, dRes=D)),
            4 * tensor_bytes)
    if "gemm" in sel:
        st2 = torch.empty(ops.nt_stat_rows(M) * 2 * C, device=dev)
        for tile in (0, 2, 3, 1):
            rep(f"gemm_nt 728x728 +stats tile={tile}", timeit(lambda: ops.gemm_nt(X, Wp, Y, M, C, C, stats=st2, tile=tile)),
                flops=2.0 * M * C * C)
        out = torch.empty(C * C, device=dev)
        for tile in (2, 1):
            rep(f"weight_grad 728x728 tile={tile}", timeit(lambda: ops.weight_grad(D, X, M, C, C, out, tile=tile)),
                flops=2.0 * M * C * C)
        rps = ops._lib.call("xcp_gemm_tn_rows_per_split", 1, 0, M, C, C, 0)
        S = (M + rps - 1) // rps
        P = torch.empty(S * C * C, device=dev)
        rep(f"gemm_tn kernel only S={S}", timeit(lambda: ops.gemm_tn(D, X, P, M, C, C, S, rps)), flops=2.0 * M * C * C)
        rep(f"reduce_slabs S={S}", timeit(lambda: ops.reduce_slabs(P, S, C * C, out)), 4 * S * C * C)
    if "ksweep" in sel:
        # NT 256x256 kernel: N = 1024 (4 column tiles), M = 64 R row tiles -> exactly R rounds of
        # 256 workgroups; time vs rounds and vs K separates the per-tile fixed cost (prologue
        # fill + epilogue) from the per-K-tile main-loop cost
        Kmax, Nn = 3072, 1024
        Xk = torch.randn(256 * 64 * 4, Kmax, device=dev, generator=g).to(dt)
        Wk = (torch.randn(Nn, Kmax, device=dev, generator=g) / 27).to(dt)
        Yk = torch.empty(256 * 64 * 4, Nn, device=dev, dtype=dt)
        for R in (1, 2, 4):
            for K in (256, 768, 1536, 3072):
                m = 256 * 64 * R
                stk = torch.empty(ops.nt_stat_rows(m) * 2 * Nn, device=dev)
                for stats in (stk, None):
                    Xv = Xk[:m].narrow(1, 0, K)
                    rep(f"nt R={R} K={K} stats={stats is not None}",
                        timeit(lambda: ops.gemm_nt(Xv, Wk.narrow(1, 0, K), Yk[:m], m, Nn, K, stats=stats, lda=Kmax,
                                                   ldb=Kmax)), flops=2.0 * m * Nn * K)
        del Xk, Wk, Yk
        # TN 256x256 kernel: 1024 x 1024 output (16 tiles) x 16 splits = 256 workgroups, rows per split swept
        for rps in (512, 1024, 2048, 4096, 8192):
            m = rps * 16
            Gt = torch.randn(m, 1024, device=dev, generator=g).to(dt)
            Xt = torch.randn(m, 1024, device=dev, generator=g).to(dt)
            P = torch.empty(16 * 1024 * 1024, device=dev)
            rep(f"tn rows/split={rps}", timeit(lambda: ops.gemm_tn(Gt, Xt, P, m, 1024, 1024, 16, rps)),
                flops=2.0 * m * 1024 * 1024)
            del Gt, Xt, P
    if "roof_ops" in sel:   # the bench's two roofline ops at the step's shape (736 pitch), for the PMC passes
        CP = 736
        Xp = torch.zeros(M, CP, device=dev, dtype=dt)
        Xp[:, :C] = X
        Yp = torch.empty_like(Xp)
        Wpp = torch.zeros(CP, CP, device=dev, dtype=dt)
        Wpp[:C, :C] = Wp
        Wtp = torch.zeros(9, CP, device=dev)
        Wtp[:, :C] = Wt
        scp, shp = torch.zeros(CP, device=dev), torch.zeros(CP, device=dev)
        scp[:C], shp[:C] = sc, sh
        stp = torch.empty(ops.nt_stat_rows(M) * 2 * CP, device=dev)
        rep("roofline op: gemm_nt 736 pitch +stats", timeit(lambda: ops.gemm_nt(Xp, Wpp, Yp, M, CP, CP, stats=stp)),
            flops=2.0 * M * C * C)
        rep("roofline op: dw_fwd 736 pitch act=2", timeit(lambda: ops.dw_fwd(2, Xp, Yp, Wtp, scp, shp, N, H, W, CP)),
            2 * (2 * M * C) + 36 * C)
    if "vendor" in sel:   # hipBLASLt (torch.matmul) on the middle-flow pointwise shape, against the xcp op
        CP = 736
        Xp = torch.zeros(M, CP, device=dev, dtype=dt)
        Xp[:, :C] = X
        Wpp = torch.zeros(CP, CP, device=dev, dtype=dt)
        Wpp[:C, :C] = Wp
        Yp = torch.empty_like(Xp)
        stp = torch.empty(ops.nt_stat_rows(M) * 2 * CP, device=dev)
        WT = Wpp.t().contiguous()
        rep("hipBLASLt torch.matmul 92416x736x736", timeit(lambda: torch.matmul(Xp, WT, out=Yp)), flops=2.0 * M * C * C)
        rep("xcp gemm_nt 92416x736x736 (no stats)", timeit(lambda: ops.gemm_nt(Xp, Wpp, Yp, M, CP, CP)), flops=2.0 * M * C * C)
        rep("xcp gemm_nt 92416x736x736 +stats", timeit(lambda: ops.gemm_nt(Xp, Wpp, Yp, M, CP, CP, stats=stp)),
            flops=2.0 * M * C * C)
        del Xp, Yp
    if "dw_after" in sel:   # the 19^2 x 736 depthwise forward alone (its input re-read every launch) against
        # right after the pointwise GEMM that writes its input (as in the step), timed by events around it only
        CP = 736
        Xp = torch.zeros(M, CP, device=dev, dtype=dt)
        Xp[:, :C] = X
        Yp, Zp = torch.empty_like(Xp), torch.empty_like(Xp)
        Wpp = torch.zeros(CP, CP, device=dev, dtype=dt)
        Wpp[:C, :C] = Wp
        Wtp = torch.zeros(9, CP, device=dev)
        Wtp[:, :C] = Wt
        scp, shp = torch.zeros(CP, device=dev), torch.zeros(CP, device=dev)
        scp[:C], shp[:C] = sc, sh
        stp = torch.empty(ops.nt_stat_rows(M) * 2 * CP, device=dev)
        ops.gemm_nt(Xp, Wpp, Yp, M, CP, CP, stats=stp)
        rep("dw_fwd 736 pitch act=2 alone", timeit(lambda: ops.dw_fwd(2, Yp, Zp, Wtp, scp, shp, N, H, W, CP)), 2 * (2 * M * C))
        evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(20)]
        for i in range(23):
            ops.gemm_nt(Xp, Wpp, Yp, M, CP, CP, stats=stp)
            if i >= 3:
                evs[i - 3][0].record()
            ops.dw_fwd(2, Yp, Zp, Wtp, scp, shp, N, H, W, CP)
            if i >= 3:
                evs[i - 3][1].record()
        torch.cuda.synchronize()
        ms = sum(a.elapsed_time(b) for a, b in evs) / len(evs)
        rep("dw_fwd 736 pitch act=2 after its GEMM", ms, 2 * (2 * M * C))
        del Xp, Yp, Zp
    if "ntprobe" in sel:   # the 256x256 NT kernel at the step's shape and at whole rounds (probe variants)
        CP = 736
        Xp = torch.zeros(M, CP, device=dev, dtype=dt)
        Xp[:, :C] = X
        Yp = torch.empty_like(Xp)
        Wpp = torch.zeros(CP, CP, device=dev, dtype=dt)
        Wpp[:C, :C] = Wp
        stp = torch.empty(ops.nt_stat_rows(M) * 2 * CP, device=dev)
        rep("nt 736 pitch +stats", timeit(lambda: ops.gemm_nt(Xp, Wpp, Yp, M, CP, CP, stats=stp)), flops=2.0 * M * C * C)
        del Xp, Yp
        Nn = 1024
        for K in (768, 3072):
            m = 256 * 64 * 4
            Xk = torch.randn(m, K, device=dev, generator=g).to(dt)
            Wk = (torch.randn(Nn, K, device=dev, generator=g) / 27).to(dt)
            Yk = torch.empty(m, Nn, device=dev, dtype=dt)
            rep(f"nt R=4 K={K}", timeit(lambda: ops.gemm_nt(Xk, Wk, Yk, m, Nn, K, tile=3)), flops=2.0 * m * Nn * K)
            del Xk, Wk, Yk
    if "sparse" in sel:   # the step's persistent-kernel shapes: auto (tile 0: sparse last round on the 128x128
        # kernel when the last round is < 3/4 full) against every row on the persistent kernel (tile 3)
        for (m, n, k, stats) in ((1401856, 256, 128, True), (1401856, 256, 256, True), (350464, 736, 256, True),
                                 (350464, 736, 736, True), (92416, 736, 736, True), (92416, 1024, 736, True),
                                 (25600, 1536, 1024, True), (25600, 2048, 1536, True), (25600, 1024, 1536, False),
                                 (25600, 1536, 2048, False), (92416, 736, 1024, False), (92416, 736, 736, False),
                                 (350464, 736, 736, False), (350464, 256, 736, False)):
            Xs = torch.randn(m, k, device=dev, generator=g).to(dt)
            Ws = (torch.randn(n, k, device=dev, generator=g) / 27).to(dt)
            Ys = torch.empty(m, n, device=dev, dtype=dt)
            sts = torch.empty(ops.nt_stat_rows(m) * 2 * n, device=dev) if stats else None
            for tile in (0, 3, 0, 3):
                rep(f"nt {m}x{n}x{k} stats={int(stats)} tile {tile}",
                    timeit(lambda: ops.gemm_nt(Xs, Ws, Ys, m, n, k, stats=sts, tile=tile)), flops=2.0 * m * n * k)
            del Xs, Ws, Ys, sts
    if "dwf_only" in sel:     # one kernel for the PMC passes
        rep("dw_fwd act=2", timeit(lambda: ops.dw_fwd(2, X, Y, Wt, sc, sh, N, H, W, C)), 2 * tensor_bytes)
    if "dwb_only" in sel:
        rep("dw_bwd act=2 +bnsums", timeit(lambda: ops.dw_bwd(2, D, X, Wt, sc, sh, Y, dW, N, H, W, C, bn_stats=st)),
            3 * tensor_bytes)
    if "nt_only" in sel:      # one kernel for the PMC passes
        st2 = torch.empty(ops.nt_stat_rows(M) * 2 * C, device=dev)
        rep("gemm_nt 728x728 +stats", timeit(lambda: ops.gemm_nt(X, Wp, Y, M, C, C, stats=st2)), flops=2.0 * M * C * C)
    if "tn_only" in sel:
        rps = ops._lib.call("xcp_gemm_tn_rows_per_split", 1, 0, M, C, C, 0)
        S = (M + rps - 1) // rps
        P = torch.empty(S * C * C, device=dev)
        rep(f"gemm_tn kernel only S={S}", timeit(lambda: ops.gemm_tn(D, X, P, M, C, C, S, rps)), flops=2.0 * M * C * C)
    if "tnshape" in sel:   # the step's weight-gradient shapes on both tiles
        for (m, n, k) in ((5531904, 128, 128), (5531904, 128, 64), (1401856, 256, 256), (1401856, 256, 128),
                          (350464, 728, 256), (350464, 728, 728), (92416, 1024, 728), (25600, 2048, 1536)):
            Gt = torch.randn(m, n, device=dev, generator=g).to(dt)
            Xt = torch.randn(m, k, device=dev, generator=g).to(dt)
            out = torch.empty(n * k, device=dev)
            for tile in (2, 1):
                rep(f"wgrad {m}x{n}x{k} tile={tile}", timeit(lambda: ops.weight_grad(Gt, Xt, m, n, k, out, tile=tile),
                                                                iters=10), 2 * m * (n + k), flops=2.0 * m * n * k)
            del Gt, Xt
    if "cold" in sel:
        flush = torch.zeros(768 * 2 ** 18, device=dev, dtype=torch.float32)   # read before each launch

        def cold(fn, iters=10):
            tot = 0.0
            for i in range(iters + 2):
                flush.sum()
                s_, e_ = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                s_.record()
                fn()
                e_.record()
                torch.cuda.synchronize()
                if i >= 2:
                    tot += s_.elapsed_time(e_)
            return tot / iters

        rep("cold copy", cold(lambda: Y.copy_(X)), 2 * tensor_bytes)
        rep("cold dw_fwd act=2", cold(lambda: ops.dw_fwd(2, X, Y, Wt, sc, sh, N, H, W, C)), 2 * tensor_bytes)
        rep("cold dw_bwd act=2 +bnsums", cold(lambda: ops.dw_bwd(2, D, X, Wt, sc, sh, Y, dW, N, H, W, C, bn_stats=st)),
            3 * tensor_bytes)
        dgm, dbt = torch.empty(C, device=dev), torch.empty(C, device=dev)
        bn = {"weight": sc, "bias": sh, "running_mean": None, "running_var": None, "eps": 1e-5, "momentum": 0.1,
              "track": False}
        rep("cold bn_backward (reduce+apply)", cold(lambda: ops.bn_backward(D, X, M, C, bn, st, Y, dgm, dbt)),
            5 * tensor_bytes)
        st2 = torch.empty(ops.nt_stat_rows(M) * 2 * C, device=dev)
        rep("cold gemm_nt 728 +stats", cold(lambda: ops.gemm_nt(X, Wp, Y, M, C, C, stats=st2)), flops=2.0 * M * C * C)
        outw = torch.empty(C * C, device=dev)
        rep("cold weight_grad 728", cold(lambda: ops.weight_grad(D, X, M, C, C, outw)), flops=2.0 * M * C * C)
        del flush
    if "blas" in sel:
        rep("hipBLASLt X @ Wp^T 728x728", timeit(lambda: torch.matmul(X, Wp.t())), flops=2.0 * M * C * C)
        rep("hipBLASLt D^T @ X 728x728", timeit(lambda: torch.matmul(D.t(), X)), flops=2.0 * M * C * C)
        X8 = torch.randn(8192, 8192, device=dev, generator=g).to(dt)
        rep("hipBLASLt 8192^3", timeit(lambda: torch.matmul(X8, X8), iters=10), flops=2.0 * 8192 ** 3)
    if "bn" in sel:
        dgm, dbt = torch.empty(C, device=dev), torch.empty(C, device=dev)
        bn = {"weight": sc, "bias": sh, "running_mean": None, "running_var": None, "eps": 1e-5, "momentum": 0.1,
              "track": False}
        rep("bn_backward (reduce+apply)", timeit(lambda: ops.bn_backward(D, X, M, C, bn, st, Y, dgm, dbt)),
            4 * tensor_bytes)
    if "chanred" in sel:   # per-channel reductions: BN forward stats (1 tensor), BN backward sums (2 tensors)
        R = ops._lib.call("xcp_chanred_parts", M, C)
        part = torch.empty(R * 2 * C, device=dev)
        rep("row_stats 19^2 x 728 (1 tensor)", timeit(lambda: ops._lib.call("xcp_row_stats", 1, ops._p(X), M, C,
                                                                            ops._p(part), ops.stream())), tensor_bytes)
        rep("bn_bwd_reduce 19^2 x 728 (2 tensors)",
            timeit(lambda: ops._lib.call("xcp_bn_bwd_reduce", 1, ops._p(D), ops._p(X), ops._p(st["mean"]),
                                         ops._p(st["invstd"]), 0, 0, M, C, ops._p(part), ops.stream())),
            2 * tensor_bytes)
    if "dwgeom" in sel:   # depthwise backward, ~92k pixels x 736 channels: walk length vs frame width
        for (Ng, Hg, Wg) in ((256, 19, 19), (33, 147, 19), (33, 19, 147), (4, 147, 147)):
            Mg = Ng * Hg * Wg
            Xg = torch.randn(Mg, 736, device=dev, generator=g).to(dt)
            Dg = torch.randn(Mg, 736, device=dev, generator=g).to(dt)
            Yg = torch.empty_like(Xg)
            Wtg = torch.randn(9, 736, device=dev, generator=g)
            scg = torch.rand(736, device=dev, generator=g) + 0.5
            shg = torch.randn(736, device=dev, generator=g)
            dWg = torch.empty(736 * 9, device=dev)
            stg = {"mean": torch.zeros(736, device=dev), "invstd": torch.ones(736, device=dev)}
            rep(f"dw_bwd N={Ng} {Hg}x{Wg} x 736 act=2", timeit(lambda: ops.dw_bwd(2, Dg, Xg, Wtg, scg, shg, Yg, dWg, Ng, Hg,
                                                                                   Wg, 736, bn_stats=stg)),
                6 * Mg * 736)
            rep(f"dw_fwd N={Ng} {Hg}x{Wg} x 736 act=2", timeit(lambda: ops.dw_fwd(2, Xg, Yg, Wtg, scg, shg, Ng, Hg, Wg,
                                                                                   736)), 4 * Mg * 736)
            del Xg, Dg, Yg
    if "poolbwd" in sel:   # max-pool backward + BN reduce of blocks 2 / 3 (74^2 x 256, 37^2 x 736)
        from xcp.engine import Stats
        for Hb, Cb in ((74, 256), (37, 736)):
            OHb = (Hb - 1) // 2 + 1
            Yb = torch.randn(N * Hb * Hb * Cb, device=dev, generator=g).to(dt)
            dOb = torch.randn(N * OHb * OHb * Cb, device=dev, generator=g).to(dt)
            amb = torch.randint(0, 9, (N * OHb * OHb * Cb,), device=dev, generator=g, dtype=torch.uint8)
            dzb = torch.empty_like(Yb)
            stb = Stats(Cb, dev)
            byts = 2 * (2 * Yb.numel() + dOb.numel()) + amb.numel()
            rep(f"maxpool_bwd_bnred {Hb}^2x{Cb}", timeit(lambda: ops.maxpool_bwd_bnred(dOb, amb, dzb, Yb, stb, N, Hb, Hb,
                                                                                      Cb)), byts)
            del Yb, dOb, amb, dzb
    if "bnapply" in sel:   # BN-backward apply at the middle-flow shape (92,416 rows x 736), without / with the mask
        Ma, Ca = N * H * W, 736
        dZa = torch.randn(Ma, Ca, device=dev, generator=g).to(dt)
        Ya = torch.randn(Ma, Ca, device=dev, generator=g).to(dt)
        dYa = torch.empty_like(Ya)
        coef = torch.randn(3 * Ca, device=dev, generator=g)
        sta = {"scale": torch.rand(Ca, device=dev, generator=g) + 0.5, "shift": torch.randn(Ca, device=dev, generator=g)}
        for relu in (False, True):
            rep(f"bn_bwd_apply {Ma}x{Ca} mask={int(relu)}",
                timeit(lambda: ops.bn_apply_coef(dZa, Ya, dYa, coef, sta, Ma, Ca, relu)), 3 * 2 * Ma * Ca)
        del dZa, Ya, dYa
    if "dwsmall" in sel:   # tiny-frame depthwise forward at the XceptionLSTMA shapes (1920 64^2 frames)
        for Hs, Cs in ((4, 736), (8, 736), (8, 256)):
            Ms = 1920 * Hs * Hs
            Xs = torch.randn(Ms, Cs, device=dev, generator=g).to(dt)
            Ys = torch.empty_like(Xs)
            Wts = torch.randn(9, Cs, device=dev, generator=g)
            scs = torch.rand(Cs, device=dev, generator=g) + 0.5
            shs = torch.randn(Cs, device=dev, generator=g)
            rep(f"dw_fwd small 1920x{Hs}^2x{Cs} act=2", timeit(lambda: ops.dw_fwd(2, Xs, Ys, Wts, scs, shs, 1920, Hs, Hs,
                                                                                   Cs)), 4 * Ms * Cs)
            del Xs, Ys
    if "tailpool" in sel:   # the three pooled block tails of the entry flow (blocks 1-3)
        for Hp, Cp in ((147, 128), (74, 256), (37, 736)):
            OHp = (Hp - 1) // 2 + 1
            Yp = torch.randn(N * Hp * Hp * Cp, device=dev, generator=g).to(dt)
            Sp = torch.randn(N * OHp * OHp * Cp, device=dev, generator=g).to(dt)
            Op = torch.empty_like(Sp)
            Ap = torch.empty(N * OHp * OHp * Cp, device=dev, dtype=torch.uint8)
            sc2 = (torch.rand(Cp, device=dev, generator=g) + 0.5)
            sh2 = torch.randn(Cp, device=dev, generator=g)
            byts = 2 * (Yp.numel() + 2 * Sp.numel()) + Ap.numel()
            rep(f"tail_fwd pooled {Hp}^2x{Cp}", timeit(lambda: ops.tail_fwd(Yp, sc2, sh2, True, Sp, sc2, sh2, Op, Ap, N, Hp,
                                                                            Hp, Cp)), byts)
            del Yp, Sp, Op, Ap
    if "pad" in sel:   # channel pitch 728 vs 736 (64-B aligned rows) vs 768 (128-B aligned) at 19^2 x 256
        for Cp in (728, 736, 768):
            Mp = N * H * W
            Xp = torch.randn(Mp, Cp, device=dev, generator=g).to(dt)
            Yp = torch.empty_like(Xp)
            Dp = torch.randn(Mp, Cp, device=dev, generator=g).to(dt)
            Wtp = torch.randn(9, Cp, device=dev, generator=g)
            scp = torch.rand(Cp, device=dev, generator=g) + 0.5
            shp = torch.randn(Cp, device=dev, generator=g)
            dWp = torch.empty(Cp * 9, device=dev)
            stp = {"mean": torch.zeros(Cp, device=dev), "invstd": torch.ones(Cp, device=dev)}
            tb = Mp * Cp * 2
            rep(f"C={Cp} dw_fwd act=2", timeit(lambda: ops.dw_fwd(2, Xp, Yp, Wtp, scp, shp, N, H, W, Cp)), 2 * tb)
            rep(f"C={Cp} dw_bwd act=2 +bnsums", timeit(lambda: ops.dw_bwd(2, Dp, Xp, Wtp, scp, shp, Yp, dWp, N, H, W, Cp,
                                                                           bn_stats=stp)), 3 * tb)
            st2 = torch.empty(ops.nt_stat_rows(Mp) * 2 * C, device=dev)
            Wq = torch.zeros(C, Cp, device=dev, dtype=dt)
            Wq[:, :C] = Wp
            rep(f"ld={Cp} gemm_nt 728x728 +stats", timeit(lambda: ops.gemm_nt(Xp, Wq, Yp, Mp, C, C, stats=st2, lda=Cp,
                                                                               ldb=Cp, ldc=Cp)), flops=2.0 * Mp * C * C)
            outp = torch.empty(C * C, device=dev)
            rep(f"ld={Cp} weight_grad 728x728", timeit(lambda: ops.weight_grad(Dp, Xp, Mp, C, C, outp, ldg=Cp, ldx=Cp)),
                flops=2.0 * Mp * C * C)
            del Xp, Yp, Dp
    if "dwshapes" in sel:   # depthwise forward at the step's shapes (256 frames)
        for (Hs, Cs, act) in ((147, 64, 0), (147, 128, 2), (74, 128, 1), (74, 256, 2), (37, 256, 1), (37, 736, 2),
                              (19, 736, 1), (19, 736, 2), (19, 1024, 2), (10, 1536, 0), (10, 2048, 2)):
            Ms = N * Hs * Hs
            Xs = torch.randn(Ms, Cs, device=dev, generator=g).to(dt)
            Ys = torch.empty_like(Xs)
            Wts = torch.randn(9, Cs, device=dev, generator=g)
            scs = torch.rand(Cs, device=dev, generator=g) + 0.5
            shs = torch.randn(Cs, device=dev, generator=g)
            rep(f"dw_fwd {Hs}^2 x {Cs} act={act}", timeit(lambda: ops.dw_fwd(act, Xs, Ys, Wts, scs, shs, N, Hs, Hs, Cs)),
                4 * Ms * Cs)
            # output fingerprint (compares kernel variants run in separate processes bit for bit)
            raw = Ys.view(torch.int16).long() if Ys.dtype == torch.bfloat16 else Ys.view(torch.int32).long()
            pos = torch.arange(raw.numel(), device=dev).view(raw.shape) % 1000003
            print(f"  fingerprint {int((raw * pos).sum())} {int(raw.sum())}", flush=True)
            del Xs, Ys, raw, pos
    if "entrygemm" in sel:   # entry-flow forward pointwise GEMMs (+BN stats) on each tile kernel
        for (Me, Ne, Ke) in ((5531904, 128, 64), (5531904, 128, 128), (1401856, 256, 128), (1401856, 256, 256),
                             (350464, 736, 256), (350464, 736, 736)):
            Ae = torch.randn(Me, Ke, device=dev, generator=g).to(dt)
            Be = (torch.randn(Ne, Ke, device=dev, generator=g) / Ke ** 0.5).to(dt)
            Ce = torch.empty(Me, Ne, device=dev, dtype=dt)
            ste = torch.empty(ops.nt_stat_rows(Me), 2, Ne, device=dev)
            for tl in (1, 2, 3, 0):
                rep(f"gemm_nt {Me}x{Ne}x{Ke} +stats tile {tl}", timeit(lambda: ops.gemm_nt(Ae, Be, Ce, Me, Ne, Ke, stats=ste,
                                                                                       tile=tl), iters=10),
                    2 * Me * (Ke + Ne), flops=2.0 * Me * Ne * Ke)
            del Ae, Be, Ce, ste
    if "dwbshapes" in sel:   # depthwise backward at the step's shapes (256 frames)
        for (Hs, Cs, act, res) in ((147, 64, 0, False), (147, 128, 2, False), (74, 128, 1, True), (74, 256, 2, False),
                                   (37, 256, 1, True), (37, 736, 2, False), (19, 736, 1, True), (19, 736, 2, False),
                                   (10, 1024, 2, False), (10, 1536, 0, False)):
            Ms = N * Hs * Hs
            Xs = torch.randn(Ms, Cs, device=dev, generator=g).to(dt)
            Ds = torch.randn(Ms, Cs, device=dev, generator=g).to(dt)
            Ys = torch.empty_like(Xs)
            Wts = torch.randn(9, Cs, device=dev, generator=g)
            scs = torch.rand(Cs, device=dev, generator=g) + 0.5
            shs = torch.randn(Cs, device=dev, generator=g)
            dWs = torch.empty(Cs * 9, device=dev)
            sts = {"mean": torch.zeros(Cs, device=dev), "invstd": torch.ones(Cs, device=dev)} if act == 2 else None
            rep(f"dw_bwd {Hs}^2 x {Cs} act={act}{' +res' if res else ''}",
                timeit(lambda: ops.dw_bwd(act, Ds, Xs, Wts, scs, shs, Ys, dWs, N, Hs, Hs, Cs, bn_stats=sts,
                                          dRes=Ds if res else None)), (4 if res else 3) * Ms * Cs * 2)
            del Xs, Ds, Ys
    if "dwloc" in sel:   # same bytes, different channel counts: channel slicing vs frame size at 19^2 and 147^2
        for (Hs, Cs, Ns) in ((19, 736, 256), (19, 128, 1472), (19, 64, 2944), (147, 128, 256), (147, 736, 44)):
            Ms = Ns * Hs * Hs
            Xs = torch.randn(Ms, Cs, device=dev, generator=g).to(dt)
            Ds = torch.randn(Ms, Cs, device=dev, generator=g).to(dt)
            Ys = torch.empty_like(Xs)
            Wts = torch.randn(9, Cs, device=dev, generator=g)
            scs = torch.rand(Cs, device=dev, generator=g) + 0.5
            shs = torch.randn(Cs, device=dev, generator=g)
            dWs = torch.empty(Cs * 9, device=dev)
            sts = {"mean": torch.zeros(Cs, device=dev), "invstd": torch.ones(Cs, device=dev)}
            rep(f"dw_fwd {Hs}^2 x {Cs} N={Ns} act=2", timeit(lambda: ops.dw_fwd(2, Xs, Ys, Wts, scs, shs, Ns, Hs, Hs, Cs)),
                4 * Ms * Cs)
            rep(f"dw_bwd {Hs}^2 x {Cs} N={Ns} act=2", timeit(lambda: ops.dw_bwd(2, Ds, Xs, Wts, scs, shs, Ys, dWs, Ns, Hs,
                                                                                 Hs, Cs, bn_stats=sts)), 6 * Ms * Cs)
            del Xs, Ds, Ys
    if "conv1" in sel:   # stem conv1 3->32 3x3 s2 at 256 frames of 299^2 (fp32 NCHW in, bf16 NHWC out)
        Xc = torch.rand(N, 3, 299, 299, device=dev, generator=g)
        Wc = torch.randn(32, 3, 3, 3, device=dev, generator=g) / 5
        Yc = torch.empty(N * 149 * 149, 32, device=dev, dtype=dt)
        byts = Xc.numel() * 4 + Yc.numel() * 2
        rep("conv1 fwd 299^2 -> 149^2 x 32", timeit(lambda: ops.conv1_fwd(Xc, Wc, Yc, N, 299, 299), iters=10), byts)

        def fwd_then_stats():
            ops.conv1_fwd(Xc, Wc, Yc, N, 299, 299)
            ops.row_stats(Yc, N * 149 * 149, 32)
        rep("conv1 fwd + bn1 row_stats pass", timeit(fwd_then_stats, iters=10), byts + Yc.numel() * 2)
        rep("conv1 fwd with bn1 stats fused", timeit(lambda: ops.conv1_fwd_stats(Xc, Wc, Yc, N, 299, 299), iters=10), byts)
        dWc = torch.empty(32 * 27, device=dev)
        rep("conv1 wgrad", timeit(lambda: ops.conv1_wgrad(Xc, Yc, dWc, N, 299, 299), iters=10), byts)
        # BN1's backward apply + ReLU mask, then the weight gradient, vs the fused form (reads dZ and y)
        Zc = torch.randn(N * 149 * 149, 32, device=dev, generator=g).to(dt)
        coef = torch.randn(96, device=dev, generator=g)
        stc = {"scale": torch.randn(32, device=dev, generator=g), "shift": torch.randn(32, device=dev, generator=g)}
        Dc = torch.empty_like(Yc)
        rows1 = N * 149 * 149
        rep("bn1 apply (dZ, y -> dC1)", timeit(lambda: ops.bn_apply_coef(Zc, Yc, Dc, coef, stc, rows1, 32, relu=True),
                                               iters=10), 3 * Yc.numel() * 2)

        def unfused():
            ops.bn_apply_coef(Zc, Yc, Dc, coef, stc, rows1, 32, relu=True)
            ops.conv1_wgrad(Xc, Dc, dWc, N, 299, 299)
        rep("bn1 apply + conv1 wgrad", timeit(unfused, iters=10), byts + 3 * Yc.numel() * 2)
        rep("conv1 wgrad with bn1 apply fused", timeit(lambda: ops.conv1_wgrad_bn(Xc, Zc, Yc, coef, stc, dWc, N, 299, 299,
                                                                                  32), iters=10),
            byts + Yc.numel() * 2)
        del Xc, Yc, Zc, Dc
    if "conv2" in sel:   # stem conv2 3x3 32->64 at 256 frames of 149^2 -> 147^2 (bf16 NHWC): fwd (+stats), dgrad, wgrad
        a1 = torch.randn(N * 149 * 149, 32, device=dev, generator=g).to(dt)
        w2 = (torch.randn(64, 9, 32, device=dev, generator=g) / 17).to(dt)
        w2t = w2.permute(2, 1, 0).contiguous()   # [32][9][64]
        c2 = torch.empty(N * 147 * 147, 64, device=dev, dtype=dt)
        R2 = ops.conv3x3_parts(0, N, 149, 149)
        st2 = torch.empty(R2 * 2 * 64, device=dev)
        byts = a1.numel() * 2 + c2.numel() * 2
        rep("conv2 fwd +stats 149^2 x 32 -> 147^2 x 64", timeit(lambda: ops.conv3x3(0, a1, w2, c2, st2, N, 149, 149),
                                                             iters=10), byts, 2.0 * c2.numel() * 288)
        dA = torch.empty_like(a1)
        rep("conv2 dgrad", timeit(lambda: ops.conv3x3(1, c2, w2t, dA, None, N, 147, 147), iters=10), byts,
            2.0 * c2.numel() * 288)
        w2g = torch.empty(64 * 288, device=dev)
        rep("conv2 wgrad (+ slab reduce)", timeit(lambda: ops.conv3x3_wgrad(c2, a1, w2g, N, 149, 149), iters=10), byts,
            2.0 * c2.numel() * 288)
        del a1, c2, dA
    if "unitbwd" in sel:   # block1 / block2 unit backward (256 frames): fused vs three kernels
        for (Hu, CO, CI) in ((147, 128, 128), (147, 128, 64), (74, 256, 256), (74, 256, 128)):
            Mu = N * Hu * Hu
            Gu = torch.randn(Mu, CO, device=dev, generator=g).to(dt)
            Yu = torch.randn(Mu, CO, device=dev, generator=g).to(dt)
            cu = torch.randn(3 * CO, device=dev, generator=g) * 0.5
            dYu = torch.empty_like(Gu)
            Wu = (torch.randn(CI, CO, device=dev, generator=g) / 11).to(dt)
            Xu = torch.randn(Mu, CI, device=dev, generator=g).to(dt)
            dDu = torch.empty(Mu, CI, device=dev, dtype=dt)
            dWu = torch.empty(CO * CI, device=dev)
            byts = 2 * Mu * (2 * CO + 2 * CI)

            def three():
                ops.bn_apply_coef(Gu, Yu, dYu, cu, None, Mu, CO)
                ops.gemm_nt(dYu, Wu, dDu, Mu, CI, CO)
                ops.weight_grad(dYu, Xu, Mu, CO, CI, dWu)

            rep(f"unit bwd {Hu}^2 {CO}->{CI} three kernels", timeit(three, iters=10), byts)
            rep(f"unit bwd {Hu}^2 {CO}->{CI} fused", timeit(lambda: ops.unit_bwd(Gu, Yu, cu, Wu, Xu, dDu, Mu, CO, CI, dWu),
                                                           iters=10), byts)
            del Gu, Yu, dYu, Xu, dDu
    if "fin" in sel:   # BN finalize from the GEMM epilogue's partial rows (forward) and the backward's
        CP = 736
        for R in (722, 2888, 90):
            part = torch.rand(R * 2 * CP, device=dev, generator=g)
            bnp = {"weight": torch.ones(CP, device=dev), "bias": torch.zeros(CP, device=dev), "track": True,
                   "running_mean": torch.zeros(CP, device=dev), "running_var": torch.ones(CP, device=dev),
                   "momentum": 0.1, "eps": 1e-3}
            out = {k: torch.empty(CP, device=dev) for k in ("mean", "invstd", "scale", "shift")}
            rep(f"bn finalize R={R} C=728/{CP}", timeit(lambda: ops.finalize_stats(part, R, 728, float(R * 128), bnp, True, out, CP),
                                                       iters=50), R * 2 * CP * 4)
            stt = {"mean": torch.zeros(CP, device=dev), "invstd": torch.ones(CP, device=dev)}
            dg, db = torch.zeros(CP, device=dev), torch.zeros(CP, device=dev)
            Yd = torch.empty(1, device=dev, dtype=dt)
            rep(f"bn bwd finalize R={R}", timeit(lambda: ops.bn_backward_coef(None, Yd, R * 128, 728, bnp, stt, dg, db,
                                                                              part=part, R=R, CP=CP), iters=50),
                R * 2 * CP * 4)
    if "tail" in sel:
        rep("tail_fwd identity", timeit(lambda: ops.tail_fwd(X, sc, sh, False, D, None, None, Y, None, N, H, W, C)),
            3 * tensor_bytes)


if __name__ == "__main__":
    main()
