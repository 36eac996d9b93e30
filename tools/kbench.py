"""Kernel micro-benchmarks at the bench's middle-flow shapes (N=256 frames of 19x19x728,
bf16) and a few others: average launch time with HIP events, achieved GB/s or TFLOP/s.

usage: python tools/kbench.py [names...]   (default: all)
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
    sel = set(sys.argv[1:])
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
    stats = torch.empty(ops.nt_stat_rows(M) * 2 * C, device=dev)
    dW = torch.empty(C * 9, device=dev)
    st = {"mean": torch.zeros(C, device=dev), "invstd": torch.ones(C, device=dev)}
    tensor_bytes = M * C * 2
    res = []

    def rep(name, ms, byts=None, flops=None):
        line = f"{name:34s} {ms * 1e3:9.1f} us"
        if byts:
            line += f"  {byts / ms / 1e6:8.1f} GB/s"
        if flops:
            line += f"  {flops / ms / 1e9:8.1f} TFLOP/s"
        print(line, flush=True)
        res.append((name, ms))

    if not sel or "copy" in sel:
        rep("torch copy (ref BW)", timeit(lambda: Y.copy_(X)), 2 * tensor_bytes)
    if "dwrow" in sel:
        for kern in [int(v) for v in os.environ.get("XCP_DWK", "2,0,1").split(",")]:
            oldk = ops._lib.call("xcp_tune", 4, kern)
            oldb = ops._lib.call("xcp_tune", 5, kern)
            for act in (1, 2):
                rep(f"dw_fwd act={act} kernel={kern}", timeit(lambda: ops.dw_fwd(act, X, Y, Wt, sc, sh, N, H, W, C)),
                    2 * tensor_bytes)
            rep(f"dw_bwd act=2 +bnsums kernel={kern}",
                timeit(lambda: ops.dw_bwd(2, D, X, Wt, sc, sh, Y, dW, N, H, W, C, bn_stats=st)), 3 * tensor_bytes)
            rep(f"dw_bwd act=1 +res kernel={kern}",
                timeit(lambda: ops.dw_bwd(1, D, X, Wt, sc, sh, Y, dW, N, H, W, C, dRes=D)), 4 * tensor_bytes)
            ops._lib.call("xcp_tune", 4, oldk)
            ops._lib.call("xcp_tune", 5, oldb)
    if not sel or "dw_fwd" in sel:
        for px in (512, 256):
            old = ops._lib.call("xcp_tune", 0, px)
            for act in (1, 2):
                rep(f"dw_fwd act={act} maxpx={px}", timeit(lambda: ops.dw_fwd(act, X, Y, Wt, sc, sh, N, H, W, C)),
                    2 * tensor_bytes)
            ops._lib.call("xcp_tune", 0, old)
    if not sel or "dw_bwd" in sel:
        for px in (256, 512):
            old = ops._lib.call("xcp_tune", 1, px)
            rep(f"dw_bwd act=2 +bnsums maxpx={px}",
                timeit(lambda: ops.dw_bwd(2, D, X, Wt, sc, sh, Y, dW, N, H, W, C, bn_stats=st)), 3 * tensor_bytes)
            rep(f"dw_bwd act=1 maxpx={px}", timeit(lambda: ops.dw_bwd(1, D, X, Wt, sc, sh, Y, dW, N, H, W, C)),
                3 * tensor_bytes)
            ops._lib.call("xcp_tune", 1, old)
    if not sel or "gemm" in sel:
        for cfg in (0, 1, 2):
            old = ops._lib.call("xcp_tune", 2, cfg)
            st2 = torch.empty(ops.nt_stat_rows(M) * 2 * C, device=dev)
            rep(f"gemm_nt 728x728 +stats cfg={cfg}", timeit(lambda: ops.gemm_nt(X, Wp, Y, M, C, C, stats=st2)),
                flops=2.0 * M * C * C)
            ops._lib.call("xcp_tune", 2, old)
        out = torch.empty(C * C, device=dev)
        for tn in (2, 1, 0):
            old = ops._lib.call("xcp_tune", 6, tn)
            rep(f"weight_grad 728x728 tn={tn}", timeit(lambda: ops.weight_grad(D, X, M, C, C, out)),
                flops=2.0 * M * C * C)
            ops._lib.call("xcp_tune", 6, old)
    if "tnshape" in sel:   # the step's weight-gradient shapes, 256-tile kernel (cfg 1) vs 128-tile (cfg 0)
        for (m, n, k) in ((5531904, 128, 128), (5531904, 128, 64), (1401856, 256, 256), (1401856, 256, 128),
                          (350464, 728, 256), (350464, 728, 728), (92416, 1024, 728), (25600, 2048, 1536)):
            Gt = torch.randn(m, n, device=dev, generator=g).to(dt)
            Xt = torch.randn(m, k, device=dev, generator=g).to(dt)
            out = torch.empty(n * k, device=dev)
            for tn in (1, 0):
                old = ops._lib.call("xcp_tune", 6, tn)
                rep(f"wgrad {m}x{n}x{k} tn={tn}", timeit(lambda: ops.weight_grad(Gt, Xt, m, n, k, out), iters=10),
                    2 * m * (n + k), flops=2.0 * m * n * k)
                ops._lib.call("xcp_tune", 6, old)
            del Gt, Xt
    if "dwent" in sel:   # entry-flow depthwise shapes
        shapes = os.environ.get("XCP_DWSHAPES")
        shapes = [tuple(int(v) for v in t.split("x")) for t in shapes.split(",")] if shapes else \
            [(256, 147, 128), (256, 147, 64), (256, 74, 256), (256, 37, 728)]
        for (n_, h_, c_) in shapes:
            m_ = n_ * h_ * h_
            Xe = torch.randn(m_, c_, device=dev, generator=g).to(dt)
            De = torch.randn(m_, c_, device=dev, generator=g).to(dt)
            Ye = torch.empty_like(Xe)
            We = torch.randn(9 * c_, device=dev, generator=g) / 3
            sce, she = torch.rand(c_, device=dev) + 0.5, torch.randn(c_, device=dev) * 0.1
            ste = {"mean": torch.zeros(c_, device=dev), "invstd": torch.ones(c_, device=dev)}
            dWe = torch.empty(9 * c_, device=dev)
            tb = m_ * c_ * 2
            for sm_ in (0, 1):
                osm = ops._lib.call("xcp_tune", 16, sm_)
                rep(f"dw_fwd act=2 {h_}^2x{c_} small={sm_}",
                    timeit(lambda: ops.dw_fwd(2, Xe, Ye, We, sce, she, n_, h_, h_, c_), iters=10), 2 * tb)
                ops._lib.call("xcp_tune", 16, osm)
            rep(f"dw_bwd act=2 +bn {h_}^2x{c_}",
                timeit(lambda: ops.dw_bwd(2, De, Xe, We, sce, she, Ye, dWe, n_, h_, h_, c_, bn_stats=ste), iters=10), 3 * tb)
            rep(f"copy {h_}^2x{c_}", timeit(lambda: Ye.copy_(Xe), iters=10), 2 * tb)
            del Xe, De, Ye
    if "poolbn" in sel:   # pooled block tail backward: max-pool gradient + BN backward
        from xcp.engine import Stats
        for (n_, h_, c_) in ((256, 147, 128), (256, 74, 256), (256, 37, 728)):
            oh_ = (h_ - 1) // 2 + 1
            m_ = n_ * h_ * h_
            Ye = torch.randn(m_, c_, device=dev, generator=g).to(dt)
            dOut = torch.randn(n_ * oh_ * oh_, c_, device=dev, generator=g).to(dt)
            amax = torch.randint(0, 9, (n_ * oh_ * oh_ * c_,), device=dev, dtype=torch.uint8)
            dZ = torch.empty(m_, c_, device=dev, dtype=dt)
            dYe = torch.empty_like(dZ)
            ste = Stats(c_, dev)
            ste.mean.zero_(); ste.invstd.fill_(1.0)
            bn = {"weight": torch.ones(c_, device=dev), "bias": torch.zeros(c_, device=dev), "running_mean": None,
                  "running_var": None, "eps": 1e-5, "momentum": 0.1, "track": False}
            dg, db = torch.empty(c_, device=dev), torch.empty(c_, device=dev)

            def two():
                ops.maxpool_bwd(dOut, amax, dZ, n_, h_, h_, c_)
                ops.bn_backward(dZ, Ye, m_, c_, bn, ste, dYe, dg, db)

            for qv in (0, 1):
                old = ops._lib.call("xcp_tune", 12, qv)
                rep(f"maxpool_bwd quad={qv} {h_}^2x{c_}", timeit(lambda: ops.maxpool_bwd(dOut, amax, dZ, n_, h_, h_, c_),
                                                                 iters=10))
                ops._lib.call("xcp_tune", 12, old)
            rep(f"maxpool_bwd + bn_bwd {h_}^2x{c_}", timeit(two, iters=10))

            def fused():
                part, R = ops.maxpool_bwd_bnred(dOut, amax, dZ, Ye, ste, n_, h_, h_, c_)
                ops.bn_backward(dZ, Ye, m_, c_, bn, ste, dYe, dg, db, part=part, R=R)

            rep(f"maxpool_bwd_bnred + apply {h_}^2x{c_}", timeit(fused, iters=10))
            rep(f"maxpool_bwd_bnred alone {h_}^2x{c_}",
                timeit(lambda: ops.maxpool_bwd_bnred(dOut, amax, dZ, Ye, ste, n_, h_, h_, c_), iters=10))
            rep(f"bn_bwd(pool, store) {h_}^2x{c_}",
                timeit(lambda: ops.bn_backward(dZ, Ye, m_, c_, bn, ste, dYe, dg, db, pool=(dOut, amax, n_, h_, h_)),
                       iters=10))
            del Ye, dZ, dYe
    if "cold" in sel:   # middle-flow kernels with the Infinity Cache / L2 flushed before every launch
        flush = torch.zeros(768 * 2 ** 18, device=dev, dtype=torch.float32)   # read (clean lines) before each launch

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
        for fr in (0, 1):
            old = ops._lib.call("xcp_tune", 13, fr)
            rep(f"cold dw_fwd act=2 frame={fr}", cold(lambda: ops.dw_fwd(2, X, Y, Wt, sc, sh, N, H, W, C)), 2 * tensor_bytes)
            rep(f"warm dw_fwd act=2 frame={fr}", timeit(lambda: ops.dw_fwd(2, X, Y, Wt, sc, sh, N, H, W, C)), 2 * tensor_bytes)
            ops._lib.call("xcp_tune", 13, old)
        for var in (1, 2, 3):
            ov = ops._lib.call("xcp_tune", 14, var)
            rep(f"warm dw_fwd frame var={var}", timeit(lambda: ops.dw_fwd(2, X, Y, Wt, sc, sh, N, H, W, C)), 2 * tensor_bytes)
            ops._lib.call("xcp_tune", 14, ov)
        for occ in (2, 3):
            oo = ops._lib.call("xcp_tune", 17, occ)
            rep(f"cold dw_bwd act=2 +bnsums occ={occ}",
                cold(lambda: ops.dw_bwd(2, D, X, Wt, sc, sh, Y, dW, N, H, W, C, bn_stats=st)), 3 * tensor_bytes)
            rep(f"warm dw_bwd act=2 +bnsums occ={occ}",
                timeit(lambda: ops.dw_bwd(2, D, X, Wt, sc, sh, Y, dW, N, H, W, C, bn_stats=st)), 3 * tensor_bytes)
            ops._lib.call("xcp_tune", 17, oo)
        for bd in ():
            ob = ops._lib.call("xcp_tune", 15, bd)
            rep(f"cold dw_bwd act=2 +bnsums bd={bd}",
                cold(lambda: ops.dw_bwd(2, D, X, Wt, sc, sh, Y, dW, N, H, W, C, bn_stats=st)), 3 * tensor_bytes)
            rep(f"cold dw_bwd act=1 +res bd={bd}", cold(lambda: ops.dw_bwd(1, D, X, Wt, sc, sh, Y, dW, N, H, W, C, dRes=D)),
                4 * tensor_bytes)
            ops._lib.call("xcp_tune", 15, ob)
        dgm, dbt = torch.empty(C, device=dev), torch.empty(C, device=dev)
        bn = {"weight": sc, "bias": sh, "running_mean": None, "running_var": None, "eps": 1e-5, "momentum": 0.1,
              "track": False}
        rep("cold bn_backward (reduce+apply)", cold(lambda: ops.bn_backward(D, X, M, C, bn, st, Y, dgm, dbt)),
            5 * tensor_bytes)
        rep("cold gemm_nt 728 +stats", cold(lambda: ops.gemm_nt(X, Wp, Y, M, C, C,
                                                              stats=torch.empty(ops.nt_stat_rows(M) * 2 * C, device=dev))),
            flops=2.0 * M * C * C)
        outw = torch.empty(C * C, device=dev)
        rep("cold weight_grad 728", cold(lambda: ops.weight_grad(D, X, M, C, C, outw)), flops=2.0 * M * C * C)
        del flush
    if "tnabl" in sel:
        out = torch.empty(C * C, device=dev)
        P = torch.empty(28 * C * C, device=dev)
        rps = ops._lib.call("xcp_gemm_tn_rows_per_split", 1, 0, M, C, C)
        S = (M + rps - 1) // rps
        for var in [int(v) for v in os.environ.get("XCP_VARS", "0,5,6").split(",")]:
            old = ops._lib.call("xcp_tune", 3, var)
            rep(f"gemm_tn kernel only S={S} var={var}", timeit(lambda: ops.gemm_tn(D, X, P, M, C, C, S, rps)),
                flops=2.0 * M * C * C)
            ops._lib.call("xcp_tune", 3, old)
        rep(f"reduce_slabs S={S}", timeit(lambda: ops.reduce_slabs(P, S, C * C, out)), 4 * S * C * C)
    if "tnwgs" in sel:
        out = torch.empty(C * C, device=dev)
        for wgs in (128, 256, 384, 512, 768):
            old = ops._lib.call("xcp_tune", 7, wgs)
            rep(f"weight_grad 728x728 wgs={wgs}", timeit(lambda: ops.weight_grad(D, X, M, C, C, out)),
                flops=2.0 * M * C * C)
            ops._lib.call("xcp_tune", 7, old)
    if "stem" in sel:
        NS, IH = 256, 299
        OH = (IH - 3) // 2 + 1
        xin = torch.rand(NS, 3, IH, IH, device=dev, generator=g)
        w1 = torch.randn(32, 3, 3, 3, device=dev, generator=g) / 5
        c1 = torch.empty(NS * OH * OH, 32, device=dev, dtype=dt)
        d1 = torch.randn(NS * OH * OH, 32, device=dev, generator=g).to(dt)
        gw = torch.empty(32 * 27, device=dev)
        byts = xin.numel() * 4 + c1.numel() * 2
        for tile in (1, 0):
            old = ops._lib.call("xcp_tune", 8, tile)
            rep(f"conv1_fwd tile={tile}", timeit(lambda: ops.conv1_fwd(xin, w1, c1, NS, IH, IH), iters=5), byts)
            rep(f"conv1_wgrad tile={tile}", timeit(lambda: ops.conv1_wgrad(xin, d1, gw, NS, IH, IH), iters=5), byts)
            ops._lib.call("xcp_tune", 8, old)
    if "conv3" in sel:
        NS, IH = 256, 149
        OH = IH - 2
        a1 = torch.randn(NS * IH * IH, 32, device=dev, generator=g).to(dt)
        w2 = (torch.randn(64, 9 * 32, device=dev, generator=g) / 17).to(dt)
        w2t = (torch.randn(32, 9 * 64, device=dev, generator=g) / 24).to(dt)
        c2 = torch.empty(NS * OH * OH, 64, device=dev, dtype=dt)
        R = ops.conv3x3_parts(0, NS, IH, IH)
        st3 = torch.empty(R * 2 * 64, device=dev)
        byts = a1.numel() * 2 + c2.numel() * 2
        for var in (0, 1):
            old = ops._lib.call("xcp_tune", 11, var)
            rep(f"conv3x3 fwd +stats var={var}", timeit(lambda: ops.conv3x3(0, a1, w2, c2, st3, NS, IH, IH)), byts,
                flops=2.0 * c2.numel() * 288)
            rep(f"conv3x3 dgrad var={var}", timeit(lambda: ops.conv3x3(1, c2, w2t, a1, None, NS, OH, OH)), byts,
                flops=2.0 * a1.numel() * 576)
            dw2 = torch.empty(64 * 288, device=dev)
            rep(f"conv3x3 wgrad var={var}", timeit(lambda: ops.conv3x3_wgrad(c2, a1, dw2, NS, IH, IH)), byts,
                flops=2.0 * c2.numel() * 288)
            ops._lib.call("xcp_tune", 11, old)
        dw2 = torch.empty(64 * 288, device=dev)
        rep("gemm_tn im2col wgrad", timeit(lambda: ops.weight_grad(c2, a1, NS * OH * OH, 64, 288, dw2,
                                                                      gather=(2, IH, IH, OH, OH, 1, 32), ldx=32)), byts,
            flops=2.0 * c2.numel() * 288)
    if "gemmv" in sel:
        for var in [int(v) for v in os.environ.get('XCP_VARS', '0,1').split(',')]:
            old = ops._lib.call("xcp_tune", 3, var)
            st2 = torch.empty(ops.nt_stat_rows(M) * 2 * C, device=dev)
            rep(f"gemm256 var={var} +stats", timeit(lambda: ops.gemm_nt(X, Wp, Y, M, C, C, stats=st2)),
                flops=2.0 * M * C * C)
            rep(f"gemm256 var={var} nostats", timeit(lambda: ops.gemm_nt(X, Wp, Y, M, C, C)), flops=2.0 * M * C * C)
            A2 = torch.randn(M, 1456, device=dev, generator=g).to(dt)
            W2 = (torch.randn(C, 1456, device=dev, generator=g) / 27).to(dt)
            rep(f"gemm256 var={var} K=1456", timeit(lambda: ops.gemm_nt(A2, W2, Y, M, C, 1456)), flops=2.0 * M * C * 1456)
            ops._lib.call("xcp_tune", 3, old)
    if "epi" in sel:
        st2 = torch.empty(ops.nt_stat_rows(M) * 2 * C, device=dev)
        for var in (0, 8, 9, 10, 4, 2, 3):
            old = ops._lib.call("xcp_tune", 3, var)
            rep(f"gemm256 var={var} +stats", timeit(lambda: ops.gemm_nt(X, Wp, Y, M, C, C, stats=st2)),
                flops=2.0 * M * C * C)
            ops._lib.call("xcp_tune", 3, old)
    if "pgrid" in sel:
        for var in (10, 0):
            old = ops._lib.call("xcp_tune", 3, var)
            for gsz in (256, 248, 240, 192, 128):
                oldg = ops._lib.call("xcp_tune", 10, gsz)
                rep(f"gemm256p var={var} grid={gsz}", timeit(lambda: ops.gemm_nt(X, Wp, Y, M, C, C)),
                    flops=2.0 * M * C * C)
                ops._lib.call("xcp_tune", 10, oldg)
            ops._lib.call("xcp_tune", 3, old)
    if "blas" in sel:
        rep("hipBLASLt X @ Wp^T 728x728", timeit(lambda: torch.matmul(X, Wp.t())), flops=2.0 * M * C * C)
        rep("hipBLASLt D^T @ X 728x728", timeit(lambda: torch.matmul(D.t(), X)), flops=2.0 * M * C * C)
        W7 = torch.randn(768, 768, device=dev, generator=g).to(dt)
        X7 = torch.randn(M, 768, device=dev, generator=g).to(dt)
        rep("hipBLASLt 768x768", timeit(lambda: torch.matmul(X7, W7.t())), flops=2.0 * M * 768 * 768)
        X8 = torch.randn(8192, 8192, device=dev, generator=g).to(dt)
        rep("hipBLASLt 8192^3", timeit(lambda: torch.matmul(X8, X8), iters=10), flops=2.0 * 8192 ** 3)
    if "gemmk" in sel:
        for cfg in (0, 2):
            old = ops._lib.call("xcp_tune", 2, cfg)
            for K2 in (128, 728, 1456):
                A2 = torch.randn(M, K2, device=dev, generator=g).to(dt)
                W2 = (torch.randn(C, K2, device=dev, generator=g) / 27).to(dt)
                st2 = torch.empty(ops.nt_stat_rows(M) * 2 * C, device=dev)
                rep(f"gemm_nt K={K2} N=728 cfg={cfg}", timeit(lambda: ops.gemm_nt(A2, W2, Y, M, C, K2, stats=st2)),
                    flops=2.0 * M * C * K2)
            rep(f"gemm_nt K=728 nostats cfg={cfg}", timeit(lambda: ops.gemm_nt(X, Wp, Y, M, C, C)),
                flops=2.0 * M * C * C)
            W3 = (torch.randn(768, C, device=dev, generator=g) / 27).to(dt)
            Y3 = torch.empty(M, 768, device=dev, dtype=dt)
            rep(f"gemm_nt K=728 N=768 cfg={cfg}", timeit(lambda: ops.gemm_nt(X, W3, Y3, M, 768, C)),
                flops=2.0 * M * 768 * C)
            ops._lib.call("xcp_tune", 2, old)
    if not sel or "bn" in sel:
        dgm, dbt = torch.empty(C, device=dev), torch.empty(C, device=dev)
        bn = {"weight": sc, "bias": sh, "running_mean": None, "running_var": None, "eps": 1e-5, "momentum": 0.1,
              "track": False}
        rep("bn_backward (reduce+apply)", timeit(lambda: ops.bn_backward(D, X, M, C, bn, st, Y, dgm, dbt)),
            4 * tensor_bytes)
    if not sel or "tail" in sel:
        rep("tail_fwd identity", timeit(lambda: ops.tail_fwd(X, sc, sh, False, D, None, None, Y, None, N, H, W, C)),
            3 * tensor_bytes)


if __name__ == "__main__":
    main()
