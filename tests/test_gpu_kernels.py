"""Per-kernel numerics on the MI355X: every xcp kernel against a plain PyTorch fp32
reference of the same op (run on the same device).  Tolerances: fp32 mode 1e-4
relative (exact-fp32 MFMA, different summation order); bf16 mode checks against
the fp32 reference of the bf16-rounded inputs with 2e-2 relative."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

DTYPES = [torch.float32, torch.bfloat16]


def tol(dt):
    return dict(rtol=1e-4, atol=1e-4) if dt == torch.float32 else dict(rtol=2e-2, atol=2e-2)


def rel_err(a, b):
    a, b = a.double(), b.double()
    return ((a - b).norm() / b.norm().clamp_min(1e-30)).item()


def nhwc(x):  # [N,C,H,W] -> [N,H,W,C] contiguous
    return x.permute(0, 2, 3, 1).contiguous()


def nchw(x):
    return x.permute(0, 3, 1, 2).contiguous()


@pytest.fixture(scope="module")
def ops(gpu):
    from xcp import ops as o
    o._lib.load()
    return o


@pytest.mark.parametrize("dt", DTYPES)
@pytest.mark.parametrize("M,N,K", [(256, 128, 64), (1000, 728, 728), (361 * 3, 1024, 728), (100, 2048, 1536),
                                   (77, 64, 288)])
def test_gemm_nt_stats(ops, gpu, dt, M, N, K):
    g = torch.Generator(device=gpu).manual_seed(M + N + K)
    A = torch.randn(M, K, device=gpu, generator=g).to(dt)
    B = torch.randn(N, K, device=gpu, generator=g).to(dt) / K ** 0.5
    C = torch.empty(M, N, device=gpu, dtype=dt)
    R = ops.nt_stat_rows(M)
    part = torch.empty(R, 2, N, device=gpu)
    ops.gemm_nt(A, B, C, M, N, K, stats=part)
    ref = A.float() @ B.float().t()
    assert rel_err(C.float(), ref) < (1e-5 if dt == torch.float32 else 1e-2)
    s = part.double().sum(0)
    Cs = C.double()
    torch.testing.assert_close(s[0], Cs.sum(0), rtol=1e-5, atol=1e-3)
    torch.testing.assert_close(s[1], (Cs * Cs).sum(0), rtol=1e-5, atol=1e-3)


@pytest.mark.parametrize("M,N,K,lda", [(256, 256, 32, 32), (1000, 728, 728, 728), (300, 2048, 1536, 1536),
                                       (77, 64, 288, 288), (513, 264, 40, 40), (92416 // 8, 728, 728, 736),
                                       (4100, 1024, 728, 1456), (46208, 728, 728, 736), (77073, 264, 40, 40),
                                       (92416, 728, 728, 728)])
@pytest.mark.parametrize("tile", [2, 0, 3])
def test_gemm_nt256_stats(ops, gpu, M, N, K, lda, tile):
    """The 256x256 8-wave bf16 kernel (tile 2: forced for every size; tile 3: its persistent form,
    one workgroup per CU walking the tiles with the next tile's first K-tile prefetched under the
    epilogue; tile 0: automatic choice, so the large shapes take it and the small ones the 128x128
    kernel, and a sparse
    last round of 256 tiles -- 46208 and 92416 rows x 728 -- goes to the 128x128 kernel with
    its rows, output and stats rows offset): ragged M / N,
    K tails (K % 32 != 0, K <= 32: a single half-depth K-tile), a row pitch wider than K, and
    the 128-row stats layout."""
    g = torch.Generator(device=gpu).manual_seed(M + N + K)
    Abuf = torch.randn(M, lda, device=gpu, generator=g).bfloat16()
    A = Abuf[:, :K]
    B = (torch.randn(N, K, device=gpu, generator=g) / K ** 0.5).bfloat16()
    C = torch.full((M, N), float("nan"), device=gpu, dtype=torch.bfloat16)
    R = ops.nt_stat_rows(M)
    part = torch.full((R, 2, N), float("nan"), device=gpu)
    ops.gemm_nt(Abuf, B, C, M, N, K, lda=lda, stats=part, tile=tile)
    torch.cuda.synchronize()
    ref = A.float() @ B.float().t()
    assert rel_err(C.float(), ref) < 1e-2
    s = part.double().sum(0)
    Cs = C.double()
    torch.testing.assert_close(s[0], Cs.sum(0), rtol=1e-5, atol=1e-3)
    torch.testing.assert_close(s[1], (Cs * Cs).sum(0), rtol=1e-5, atol=1e-3)
    # the partial of rows [128r, 128r+128) is row r
    r = (M - 1) // 128
    torch.testing.assert_close(part[r, 0].double(), Cs[128 * r:].sum(0), rtol=1e-5, atol=1e-3)


@pytest.mark.parametrize("M,N,K,lda", [(1_401_856, 256, 128, 128), (1_401_856, 256, 256, 256),
                                       (350_464, 736, 256, 256), (5_531_904 // 4, 128, 128, 128)])
def test_gemm_nt_entry_flow_shapes_vs_fp64(ops, gpu, M, N, K, lda):
    """The entry-flow forward pointwise GEMMs of the bench step (256 frames: 74^2 x 128->256,
    74^2 x 256->256, 37^2 x 256->736 pitch; and a 147^2 x 128->128 slice) under the automatic
    tile choice (tile 0: since round 3 the persistent 256x256 kernel + the sparse-round 128x128
    tail for outputs >= 256 wide) and pinned to the 128x128 kernel (tile 1), against an fp64
    product of the same bf16 operands:
      C: every element is one of the two bf16 neighbours of the fp64 value (fp32 accumulation
         error is far below a bf16 ulp), and >= 99 % are the round-to-nearest one;
      BN partial sums (the epilogue's per-128-row sum / sum of squares of the stored bf16 C):
         equal to an fp64 sum of the stored C to fp32 summation error, and the two tiles' column
         sums agree with each other and with the fp64 product's to bf16 rounding noise."""
    g = torch.Generator(device=gpu).manual_seed(M + N + K)
    A = (torch.rand(M, lda, device=gpu, generator=g) - 0.25).bfloat16()   # post-ReLU-like, nonzero mean
    B = (torch.randn(N, K, device=gpu, generator=g) / K ** 0.5).bfloat16()
    ref = A[:, :K].double() @ B.double().t()
    rb = ref.to(torch.bfloat16).double()
    # bf16 spacing at |ref|, plus a rigorous fp32 accumulation bound (K u32 sum|a||b|) for the
    # elements whose value nearly cancels
    lim = (ref.abs().clamp_min(1e-30).log2().floor() - 7).exp2()
    lim += (A[:, :K].float().abs() @ B.float().abs().t()).double() * (K * 2.0 ** -24)
    R = ops.nt_stat_rows(M)
    sums = {}
    for tile in (0, 1):
        C = torch.full((M, N), float("nan"), device=gpu, dtype=torch.bfloat16)
        part = torch.full((R, 2, N), float("nan"), device=gpu)
        ops.gemm_nt(A, B, C, M, N, K, lda=lda, stats=part, tile=tile)
        torch.cuda.synchronize()
        Cd = C.double()
        assert not torch.isnan(Cd).any()
        d = (Cd - ref).abs()
        assert (d <= lim * 1.0001).all(), (tile, (d / lim).max().item())
        nearest = (Cd == rb).double().mean().item()
        assert nearest >= 0.99, (tile, nearest)
        s = part.double().sum(0)
        torch.testing.assert_close(s[0], Cd.sum(0), rtol=1e-5, atol=1e-5 * Cd.abs().sum(0).max().item())
        torch.testing.assert_close(s[1], (Cd * Cd).sum(0), rtol=1e-5, atol=1e-3)
        sums[tile] = s
        del C, part, Cd, d
    # the stats of the two kernels: same stored values up to the 1 % of elements rounded the other way
    scale0 = (ref.abs().sum(0) * 2.0 ** -8)
    assert ((sums[0][0] - sums[1][0]).abs() <= scale0 * 0.05 + 1e-6).all()
    assert ((sums[0][0] - ref.sum(0)).abs() <= scale0 * 0.05 + 1e-6).all()
    torch.testing.assert_close(sums[0][1], (ref * ref).sum(0), rtol=2e-3, atol=0)


@pytest.mark.parametrize("dt", DTYPES)
def test_gemm_nt_strided_gather(ops, gpu, dt):
    N, H, W, Cin, Cout = 3, 37, 37, 256, 728
    x = torch.randn(N, Cin, H, W, device=gpu).to(dt)
    w = torch.randn(Cout, Cin, 1, 1, device=gpu) / Cin ** 0.5
    ref = F.conv2d(x.float(), w, stride=2)
    OH, OW = ref.shape[2:]
    Y = torch.empty(N * OH * OW, Cout, device=gpu, dtype=dt)
    ops.gemm_nt(nhwc(x), w.reshape(Cout, Cin).to(dt).contiguous(), Y, N * OH * OW, Cout, Cin, lda=Cin,
                gather=(1, H, W, OH, OW, 2, 0))
    assert rel_err(nchw(Y.view(N, OH, OW, Cout)).float(), ref) < (1e-5 if dt == torch.float32 else 1e-2)


@pytest.mark.parametrize("dt", DTYPES)
def test_gemm_im2col_conv2_fwd_and_dgrad(ops, gpu, dt):
    N, H, W = 2, 21, 19
    x = torch.randn(N, 32, H, W, device=gpu).to(dt)
    w = (torch.randn(64, 32, 3, 3, device=gpu) / 17).requires_grad_(True)
    xr = x.float().requires_grad_(True)
    ref = F.conv2d(xr, w)
    OH, OW = H - 2, W - 2
    wp = w.detach().permute(0, 2, 3, 1).reshape(64, 288).to(dt).contiguous()
    Y = torch.empty(N * OH * OW, 64, device=gpu, dtype=dt)
    ops.gemm_nt(nhwc(x), wp, Y, N * OH * OW, 64, 288, lda=32, gather=(2, H, W, OH, OW, 1, 32))
    assert rel_err(nchw(Y.view(N, OH, OW, 64)).float(), ref) < (1e-5 if dt == torch.float32 else 1e-2)
    dy = torch.randn_like(ref).to(dt)
    ref.backward(dy.float())
    wt = w.detach().permute(1, 2, 3, 0).reshape(32, 576).to(dt).contiguous()
    dX = torch.empty(N * H * W, 32, device=gpu, dtype=dt)
    ops.gemm_nt(nhwc(dy), wt, dX, N * H * W, 32, 576, lda=64, gather=(3, H, W, OH, OW, 1, 64))
    assert rel_err(nchw(dX.view(N, H, W, 32)).float(), xr.grad) < (1e-5 if dt == torch.float32 else 1e-2)
    # weight gradient via im2col TN gather, k = tap*32 + ci
    wg = torch.empty(64 * 288, device=gpu)
    ops.weight_grad(nhwc(dy), nhwc(x), N * OH * OW, 64, 288, wg, gather=(2, H, W, OH, OW, 1, 32), ldx=32)
    wg = wg.view(64, 3, 3, 32).permute(0, 3, 1, 2)
    assert rel_err(wg, w.grad) < (1e-5 if dt == torch.float32 else 1e-2)


@pytest.mark.parametrize("dt", DTYPES)
@pytest.mark.parametrize("M,N,K", [(5000, 128, 64), (92416 // 16, 728, 728), (300, 2048, 1536), (33, 512, 2048),
                                   (1000, 264, 136), (7777, 1024, 728)])
@pytest.mark.parametrize("tile", [2, 1, 0], ids=["tn256", "tn128", "auto"])
def test_gemm_tn(ops, gpu, dt, M, N, K, tile):
    """Weight gradient (split-K slabs + column reduce) on both tiles, and the accumulate form
    (out += G^T X, gradient accumulation into param.grad)."""
    g = torch.Generator(device=gpu).manual_seed(M)
    G = torch.randn(M, N, device=gpu, generator=g).to(dt)
    X = torch.randn(M, K, device=gpu, generator=g).to(dt)
    out = torch.empty(N * K, device=gpu)
    ops.weight_grad(G, X, M, N, K, out, tile=tile)
    ref = G.float().t() @ X.float()
    assert rel_err(out.view(N, K), ref) < (1e-5 if dt == torch.float32 else 1e-3)
    base = torch.randn(N * K, device=gpu, generator=g)
    acc = base.clone()
    ops.weight_grad(G, X, M, N, K, acc, tile=tile, accumulate=True)
    assert rel_err(acc.view(N, K), ref + base.view(N, K)) < (1e-5 if dt == torch.float32 else 1e-3)


@pytest.mark.parametrize("M,N,K", [(92416, 728, 728), (20000, 1024, 736), (9000, 256, 512)])
def test_gemm_tn_xcd_align_bitwise(ops, gpu, monkeypatch, M, N, K):
    """Whole weight-gradient splits per XCD (XCP_TN_XCD_ALIGN=1: padded grid, another workgroup ->
    (split, tile) map) computes every split's slab in the same order: slabs bitwise equal."""
    g = torch.Generator(device=gpu).manual_seed(M + N)
    G = torch.randn(M, N, device=gpu, generator=g).bfloat16()
    X = torch.randn(M, K, device=gpu, generator=g).bfloat16()
    rps = ops._lib.call("xcp_gemm_tn_rows_per_split", 1, 0, M, N, K, 0)
    S = (M + rps - 1) // rps
    outs = []
    for v in ("0", "1"):
        monkeypatch.setenv("XCP_TN_XCD_ALIGN", v)
        P = torch.full((S * N * K,), float("nan"), device=gpu)
        ops.gemm_tn(G, X, P, M, N, K, S, rps)
        torch.cuda.synchronize()
        outs.append(P)
    assert not torch.isnan(outs[1]).any()
    assert torch.equal(outs[0], outs[1])
    ref = G.float().t() @ X.float()
    assert rel_err(outs[1].view(S, N, K).sum(0), ref) < 1e-3


@pytest.mark.parametrize("S,L", [(1, 5), (3, 1001), (28, 728 * 728), (768, 728 * 9), (2560, 128 * 9), (40, 2304),
                                 (17, 6), (300, 7)])
@pytest.mark.parametrize("accumulate", [False, True])
def test_reduce_slabs(ops, gpu, S, L, accumulate):
    """Slab reduction (one pass, and two levels when S is large and L small; float4 and
    scalar lanes): fp64 sums rounded once, so it matches the fp64 column sum to fp32
    rounding (once per level: atol grows with sqrt(S)); a second run is bit-identical
    (deterministic order)."""
    g = torch.Generator(device=gpu).manual_seed(S * 7 + L)
    P = torch.randn(S, L, device=gpu, generator=g)
    base = torch.randn(L, device=gpu, generator=g)
    out = base.clone() if accumulate else torch.empty(L, device=gpu)
    ops.reduce_slabs(P, S, L, out, accumulate)
    ref = P.double().sum(0) + (base.double() if accumulate else 0)
    torch.testing.assert_close(out.double(), ref, rtol=2e-6, atol=2e-6 * max(1.0, S ** 0.5))
    again = base.clone() if accumulate else torch.empty(L, device=gpu)
    ops.reduce_slabs(P, S, L, again, accumulate)
    assert torch.equal(out, again)


@pytest.mark.parametrize("CO,CI", [(128, 128), (128, 64), (256, 128), (256, 256)])
@pytest.mark.parametrize("M", [1000, 64 * 7 + 5, 150001, 5531904 // 16])
def test_unit_bwd_fused(ops, gpu, M, CO, CI):
    """Fused BN-apply + pointwise dgrad + wgrad (csrc/unitbwd.hip) against the three-kernel
    sequence it replaces (bn_bwd_apply -> dY, then dY Wt^T and dY^T X in fp32): ragged tiles and
    splits; dD within bf16 output rounding, the weight gradient to fp32 summation order; the
    accumulate form."""
    g = torch.Generator(device=gpu).manual_seed(M + CO + CI)
    G = torch.randn(M, CO, device=gpu, generator=g).bfloat16()
    Y = torch.randn(M, CO, device=gpu, generator=g).bfloat16()
    coef = torch.randn(3 * CO, device=gpu, generator=g) * 0.5
    Wt = (torch.randn(CI, CO, device=gpu, generator=g) / CO ** 0.5).bfloat16()
    X = torch.randn(M, CI, device=gpu, generator=g).bfloat16()
    dY = torch.empty(M, CO, device=gpu, dtype=torch.bfloat16)
    ops.bn_apply_coef(G, Y, dY, coef, None, M, CO)
    dD_ref = dY.float() @ Wt.float().t()
    dW_ref = dY.float().t() @ X.float()
    dD = torch.full((M, CI), float("nan"), device=gpu, dtype=torch.bfloat16)
    dW = torch.empty(CO * CI, device=gpu)
    ops.unit_bwd(G, Y, coef, Wt, X, dD, M, CO, CI, dW)
    torch.cuda.synchronize()
    assert rel_err(dD.float(), dD_ref) < 5e-3
    assert (dD.float() - dD_ref).abs().max().item() <= 2e-2 * dD_ref.abs().max().item()
    assert rel_err(dW.view(CO, CI), dW_ref) < 1e-5
    base = torch.randn(CO * CI, device=gpu, generator=g)
    acc = base.clone()
    ops.unit_bwd(G, Y, coef, Wt, X, dD, M, CO, CI, acc, accumulate=True)
    assert rel_err(acc.view(CO, CI), dW_ref + base.view(CO, CI)) < 1e-5


def test_gemm_operands_over_2gb_global_address_path(ops, gpu):
    """Operands spanning more than 2 GB take the 64-bit global-address LDS-DMA form of the
    256x256 kernels (the 32-bit buffer-offset form covers the rest): NT and TN at
    M = 1.5M rows x 728 channels (2.18 GB per operand) against fp32 torch on sampled rows /
    the full weight gradient."""
    M, C = 1_500_000, 728
    g = torch.Generator(device=gpu).manual_seed(7)
    X = (torch.rand(M, C, device=gpu, generator=g) - 0.5).to(torch.bfloat16)
    W = ((torch.rand(C, C, device=gpu, generator=g) - 0.5) / 8).to(torch.bfloat16)
    Y = torch.empty(M, C, device=gpu, dtype=torch.bfloat16)
    ops.gemm_nt(X, W, Y, M, C, C, tile=2)
    rows = torch.cat([torch.arange(0, 512, device=gpu), torch.arange(M - 512, M, device=gpu),
                      torch.randint(0, M, (2048,), device=gpu, generator=g)])
    ref = X[rows].float() @ W.float().t()
    assert rel_err(Y[rows].float(), ref) < 1e-2
    del Y
    out = torch.empty(C * C, device=gpu)
    ops.weight_grad(X, X, M, C, C, out, tile=2)
    ref = torch.zeros(C, C, device=gpu)
    for i in range(0, M, 250_000):
        xs = X[i:i + 250_000].float()
        ref += xs.t() @ xs
    assert rel_err(out.view(C, C), ref) < 1e-3


@pytest.mark.parametrize("dt", DTYPES)
@pytest.mark.parametrize("act", [0, 1, 2])
@pytest.mark.parametrize("N,C,H", [(2, 64, 37), (3, 728, 19), (2, 1536, 10), (1, 128, 9), (1, 64, 147), (2, 256, 74),
                                   (5, 728, 3), (2, 200, 1), (3, 728, 7), (4, 1024, 3), (301, 728, 19),
                                   (2600, 64, 9)])
def test_dw_fwd_bwd(ops, gpu, dt, act, N, C, H):
    """Tile forward (LDS halo tile), tiny-frame forward (W <= 8, bf16: the (7, 8), (3, 4),
    (1, 2) frames), and the fused LDS row-walk backward (dgrad + wgrad + BN partial sums).
    N = 301 / 2600: grids of more than one round of resident workgroups / waves."""
    W = H + 1
    g = torch.Generator(device=gpu).manual_seed(C + H + act)
    x = torch.randn(N, C, H, W, device=gpu, generator=g).to(dt)
    w = (torch.randn(C, 1, 3, 3, device=gpu, generator=g) / 3).requires_grad_(True)
    sc = torch.rand(C, device=gpu, generator=g) + 0.5
    sh = torch.randn(C, device=gpu, generator=g) * 0.2
    xr = x.float().requires_grad_(True)
    if act == 0:
        a = xr
    elif act == 1:
        a = F.relu(xr)
    else:
        a = F.relu(xr * sc.view(1, C, 1, 1) + sh.view(1, C, 1, 1))
    a.retain_grad()
    ref = F.conv2d(a, w, None, 1, 1, 1, C)
    Wt = w.detach().reshape(C, 9).t().contiguous()
    Y = torch.empty(N * H * W, C, device=gpu, dtype=dt)
    ops.dw_fwd(act, nhwc(x), Y, Wt, sc, sh, N, H, W, C)
    assert rel_err(nchw(Y.view(N, H, W, C)).float(), ref) < (1e-6 if dt == torch.float32 else 1e-2)
    dy = torch.randn(ref.shape, device=gpu, generator=g).to(dt)
    ref.backward(dy.float())
    # kernel output = gradient w.r.t. the transform's output (BN output for act 2) after the ReLU mask
    if act == 0:
        want = xr.grad
    elif act == 1:
        want = xr.grad
    else:
        z = xr.detach() * sc.view(1, C, 1, 1) + sh.view(1, C, 1, 1)
        want = a.grad * (z > 0)
    dX = torch.empty(N * H * W, C, device=gpu, dtype=dt)
    dW = torch.empty(C * 9, device=gpu)
    st = None
    if act == 2:
        st = {"mean": torch.randn(C, device=gpu, generator=g) * 0.1, "invstd": torch.rand(C, device=gpu, generator=g) + 0.5}
    bnpart, P = ops.dw_bwd(act, nhwc(dy), nhwc(x), Wt, sc, sh, dX, dW, N, H, W, C, bn_stats=st)
    dXn = nchw(dX.view(N, H, W, C)).float()
    assert rel_err(dXn, want) < (1e-6 if dt == torch.float32 else 1e-2)
    assert rel_err(dW.view(C, 1, 3, 3), w.grad) < (1e-5 if dt == torch.float32 else 1e-2)
    dW2 = torch.ones(C * 9, device=gpu)   # accumulate form: dW2 = 1 + dW
    ops.dw_bwd(act, nhwc(dy), nhwc(x), Wt, sc, sh, dX, dW2, N, H, W, C, accumulate=True)
    torch.testing.assert_close(dW2, dW + 1, rtol=1e-6, atol=1e-6)
    if act == 2:
        sums = bnpart.view(P, 2, C).double().sum(0)
        zhat = (x.float() - st["mean"].view(1, C, 1, 1)) * st["invstd"].view(1, C, 1, 1)
        torch.testing.assert_close(sums[0], dXn.double().sum((0, 2, 3)), rtol=1e-4, atol=1e-3)
        torch.testing.assert_close(sums[1], (dXn * zhat).double().sum((0, 2, 3)), rtol=1e-4, atol=1e-3)


@pytest.mark.parametrize("bands", [2, 3])
@pytest.mark.parametrize("N,C,H,act,res,skip", [(64, 736, 19, 2, False, False), (64, 736, 19, 1, True, False),
                                                (16, 256, 37, 2, False, False), (8, 128, 15, 1, True, True),
                                                (32, 1536, 10, 0, False, False), (5, 64, 7, 2, False, False)])
def test_dw_bwd_row_bands(ops, gpu, monkeypatch, bands, N, C, H, act, res, skip):
    """The backward's row walk split into row bands (XCP_DW_BWD_BANDS; a band re-reads the dY
    rows above and below it): dX bitwise equal to the one-band walk (the same per-pixel sums), the
    weight gradient and the BN partial sums equal to fp32 summation order (more partial rows); the
    XCD-aware workgroup order (XCP_DW_BWD_XCD) changes nothing but placement: bitwise equal."""
    W = H
    g = torch.Generator(device=gpu).manual_seed(N + C + H)
    dt = torch.bfloat16
    x = torch.randn(N * H * W, C, device=gpu, generator=g).to(dt)
    dy = torch.randn(N * H * W, C, device=gpu, generator=g).to(dt)
    Wt = torch.randn(9, C, device=gpu, generator=g) / 3
    sc = torch.rand(C, device=gpu, generator=g) + 0.5
    sh = torch.randn(C, device=gpu, generator=g) * 0.2
    dR = torch.randn(N * H * W, C, device=gpu, generator=g).to(dt) if res else None
    OH = (H - 1) // 2 + 1
    dS = torch.randn(N * OH * OH, C, device=gpu, generator=g).to(dt) if skip else None
    st = {"mean": torch.randn(C, device=gpu, generator=g) * 0.1,
          "invstd": torch.rand(C, device=gpu, generator=g) + 0.5} if act == 2 else None
    outs = []
    for b, xcd in ((1, "0"), (bands, "0"), (bands, "1")):
        monkeypatch.setenv("XCP_DW_BWD_BANDS", str(b))
        monkeypatch.setenv("XCP_DW_BWD_XCD", xcd)
        dX = torch.full((N * H * W, C), float("nan"), device=gpu, dtype=dt)
        dW = torch.empty(C * 9, device=gpu)
        bnpart, P = ops.dw_bwd(act, dy, x, Wt, sc, sh, dX, dW, N, H, W, C, dRes=dR, dSkip=dS,
                               skip_geom=(OH, OH, 2) if skip else (0, 0, 1), bn_stats=st)
        torch.cuda.synchronize()
        sums = bnpart.view(P, 2, C).double().sum(0) if bnpart is not None else None
        outs.append((dX, dW, sums, P))
    assert outs[1][3] == outs[0][3] * bands
    assert torch.equal(outs[0][0], outs[1][0])
    assert rel_err(outs[1][1], outs[0][1]) < 1e-5   # fp32 sums over more, shorter partial rows
    if act == 2:
        assert rel_err(outs[1][2], outs[0][2]) < 1e-5
    # the XCD-aware walk order is a permutation of the same waves: every output bitwise equal
    assert torch.equal(outs[2][0], outs[1][0]) and torch.equal(outs[2][1], outs[1][1])
    if act == 2:
        assert torch.equal(outs[2][2], outs[1][2])


@pytest.mark.parametrize("N,C,H,act,res", [(64, 736, 19, 2, False), (16, 256, 37, 2, False), (4, 128, 74, 1, False),
                                           (32, 1536, 10, 0, False), (64, 736, 19, 1, True)])
def test_dw_bwd_ring_read_forms(ops, gpu, monkeypatch, N, C, H, act, res):
    """Ring reads by inline asm (XCP_DW_BWD_ASM=1) or plain C++ reads (the default): the same
    arithmetic on the same values, every output bitwise equal."""
    W = H
    g = torch.Generator(device=gpu).manual_seed(3 * N + C + H)
    dt = torch.bfloat16
    x = torch.randn(N * H * W, C, device=gpu, generator=g).to(dt)
    dy = torch.randn(N * H * W, C, device=gpu, generator=g).to(dt)
    Wt = torch.randn(9, C, device=gpu, generator=g) / 3
    sc = torch.rand(C, device=gpu, generator=g) + 0.5
    sh = torch.randn(C, device=gpu, generator=g) * 0.2
    dR = torch.randn(N * H * W, C, device=gpu, generator=g).to(dt) if res else None
    st = {"mean": torch.randn(C, device=gpu, generator=g) * 0.1,
          "invstd": torch.rand(C, device=gpu, generator=g) + 0.5} if act == 2 else None
    outs = []
    for form in ("0", "1"):
        monkeypatch.setenv("XCP_DW_BWD_ASM", form)
        dX = torch.full((N * H * W, C), float("nan"), device=gpu, dtype=dt)
        dW = torch.empty(C * 9, device=gpu)
        bnpart, P = ops.dw_bwd(act, dy, x, Wt, sc, sh, dX, dW, N, H, W, C, dRes=dR, bn_stats=st)
        torch.cuda.synchronize()
        outs.append((dX, dW, bnpart.clone() if bnpart is not None else None))
    assert not torch.isnan(outs[1][0].float()).any()
    assert torch.equal(outs[0][0], outs[1][0]) and torch.equal(outs[0][1], outs[1][1])
    if act == 2:
        assert torch.equal(outs[0][2], outs[1][2])


@pytest.mark.parametrize("dt", DTYPES)
@pytest.mark.parametrize("N", [2, 701])
def test_dw_bwd_residual_and_skip(ops, gpu, dt, N):
    """Residual and strided-skip gradient adds (N = 701: several rounds of resident waves)."""
    C, H, W = 128, 15, 15
    x = torch.randn(N, C, H, W, device=gpu).to(dt)
    w = torch.randn(C, 1, 3, 3, device=gpu) / 3
    Wt = w.reshape(C, 9).t().contiguous()
    dy = torch.randn(N, C, H, W, device=gpu).to(dt)
    res = torch.randn(N, C, H, W, device=gpu).to(dt)
    OH, OW = (H - 1) // 2 + 1, (W - 1) // 2 + 1
    sk = torch.randn(N, C, OH, OW, device=gpu).to(dt)
    base = torch.empty(N * H * W, C, device=gpu, dtype=dt)
    dW = torch.empty(C * 9, device=gpu)
    ops.dw_bwd(1, nhwc(dy), nhwc(x), Wt, None, None, base, dW, N, H, W, C)
    out = torch.empty_like(base)
    ops.dw_bwd(1, nhwc(dy), nhwc(x), Wt, None, None, out, dW, N, H, W, C, dRes=nhwc(res), dSkip=nhwc(sk),
               skip_geom=(OH, OW, 2))
    want = nchw(base.view(N, H, W, C)).float() + res.float()
    want[:, :, ::2, ::2] += sk.float()
    assert rel_err(nchw(out.view(N, H, W, C)).float(), want) < (1e-6 if dt == torch.float32 else 1e-2)


@pytest.mark.parametrize("dt", DTYPES)
@pytest.mark.parametrize("act", [1, 2])
@pytest.mark.parametrize("N,C,H", [(3, 128, 15), (701, 64, 19), (256, 736, 19), (4, 200, 7)])
def test_dw_bwd_resbn(ops, gpu, dt, act, N, C, H):
    """Identity-skip block boundary (xcp_dw_bwd_resbn): the BN partial sums are taken over the final
    dX (after the residual add, as stored) against zhat = (Yb - mean) * invstd of the BN that produced
    the previous block's output; dX and dW equal the plain residual backward's."""
    W = H
    g = torch.Generator(device=gpu).manual_seed(N + C + H + act)
    x = torch.randn(N, C, H, W, device=gpu, generator=g).to(dt)
    w = torch.randn(C, 1, 3, 3, device=gpu, generator=g) / 3
    Wt = w.reshape(C, 9).t().contiguous()
    sc = torch.rand(C, device=gpu, generator=g) + 0.5
    sh = torch.randn(C, device=gpu, generator=g) * 0.2
    dy = torch.randn(N, C, H, W, device=gpu, generator=g).to(dt)
    res = torch.randn(N, C, H, W, device=gpu, generator=g).to(dt)
    yb = torch.randn(N, C, H, W, device=gpu, generator=g).to(dt)
    st = {"mean": torch.randn(C, device=gpu, generator=g) * 0.1, "invstd": torch.rand(C, device=gpu, generator=g) + 0.5}
    base = torch.empty(N * H * W, C, device=gpu, dtype=dt)
    dW0 = torch.empty(C * 9, device=gpu)
    ops.dw_bwd(act, nhwc(dy), nhwc(x), Wt, sc, sh, base, dW0, N, H, W, C, dRes=nhwc(res))
    out = torch.empty_like(base)
    dW = torch.empty(C * 9, device=gpu)
    bnpart, P = ops.dw_bwd(act, nhwc(dy), nhwc(x), Wt, sc, sh, out, dW, N, H, W, C, dRes=nhwc(res), bn_stats=st,
                           res_bn_input=nhwc(yb))
    assert torch.equal(out, base)
    torch.testing.assert_close(dW, dW0, rtol=0, atol=0)
    sums = bnpart.view(P, 2, C).double().sum(0)
    dX = out.view(N, H, W, C).double()
    zhat = (yb.permute(0, 2, 3, 1).double() - st["mean"].double()) * st["invstd"].double()
    torch.testing.assert_close(sums[0], dX.sum((0, 1, 2)), rtol=1e-4, atol=1e-3)
    torch.testing.assert_close(sums[1], (dX * zhat).sum((0, 1, 2)), rtol=1e-4, atol=1e-3)
    with pytest.raises(Exception):   # needs the residual input
        ops.dw_bwd(act, nhwc(dy), nhwc(x), Wt, sc, sh, out, dW, N, H, W, C, bn_stats=st, res_bn_input=nhwc(yb))


@pytest.mark.parametrize("dt", DTYPES)
@pytest.mark.parametrize("N,H", [(3, 15), (256, 147)])
def test_dw_bwd_skip_pre_bnrelu(ops, gpu, dt, N, H):
    """Block1 with the stem's BN2 + ReLU applied on load (engine): the rep's depthwise conv and
    the stride-2 skip conv both read a = relu(bn(x)), so the skip gradient passes the same ReLU
    mask and enters the BN partial sums (skip_pre); the skip's input is the strided activation
    (xcp_bn_act_strided).  Against torch autograd through relu(x*sc+sh) in fp32."""
    C, W = 64, H
    g = torch.Generator(device=gpu).manual_seed(N + H)
    x = torch.randn(N, C, H, W, device=gpu, generator=g).to(dt)
    w = torch.randn(C, 1, 3, 3, device=gpu, generator=g) / 3
    Wt = w.reshape(C, 9).t().contiguous()
    sc = torch.rand(C, device=gpu, generator=g) + 0.5
    sh = torch.randn(C, device=gpu, generator=g) * 0.2
    OH, OW = (H - 1) // 2 + 1, (W - 1) // 2 + 1
    # strided activation
    xs = torch.empty(N * OH * OW, C, device=gpu, dtype=dt)
    ops.bn_act_strided(nhwc(x), xs, sc, sh, True, N, H, W, OH, OW, 2, C)
    # z rounded once, as the kernels' fma (x*sc + sh in fp32 rounds twice and flips ReLU masks)
    z = (x.double() * sc.double().view(1, C, 1, 1) + sh.double().view(1, C, 1, 1)).float()
    want_s = F.relu(z)[:, :, ::2, ::2].to(dt).float()
    assert rel_err(nchw(xs.view(N, OH, OW, C)).float(), want_s) < 1e-6
    # backward with the skip gradient before the mask
    zr = z.clone().requires_grad_(True)
    a = F.relu(zr)
    dy = torch.randn(N, C, H, W, device=gpu, generator=g).to(dt)
    dsk = torch.randn(N, C, OH, OW, device=gpu, generator=g).to(dt)
    ((F.conv2d(a, w, None, 1, 1, 1, C) * dy.float()).sum() + (a[:, :, ::2, ::2] * dsk.float()).sum()).backward()
    st = {"mean": torch.randn(C, device=gpu, generator=g) * 0.1, "invstd": torch.rand(C, device=gpu, generator=g) + 0.5}
    dX = torch.empty(N * H * W, C, device=gpu, dtype=dt)
    dW = torch.empty(C * 9, device=gpu)
    bnpart, P = ops.dw_bwd(2, nhwc(dy), nhwc(x), Wt, sc, sh, dX, dW, N, H, W, C, dSkip=nhwc(dsk), skip_geom=(OH, OW, 2),
                           bn_stats=st, skip_pre=True)
    dXn = nchw(dX.view(N, H, W, C)).float()
    assert rel_err(dXn, zr.grad) < (1e-6 if dt == torch.float32 else 1e-2)
    sums = bnpart.view(P, 2, C).double().sum(0)
    zhat = (x.float() - st["mean"].view(1, C, 1, 1)) * st["invstd"].view(1, C, 1, 1)
    torch.testing.assert_close(sums[0], dXn.double().sum((0, 2, 3)), rtol=1e-4, atol=1e-3)
    torch.testing.assert_close(sums[1], (dXn * zhat).double().sum((0, 2, 3)), rtol=1e-4, atol=1e-2)


@pytest.mark.parametrize("relu", [False, True])
@pytest.mark.parametrize("dt", DTYPES)
@pytest.mark.parametrize("rows,C", [(100000, 128), (3 * 361, 728), (50, 2048)])
def test_bn_forward_backward(ops, gpu, dt, rows, C, relu):
    """BN statistics / running buffers, apply, and backward; relu=True: the gradient
    arrives for relu(bn(y)) (stem, Xception.py:170/:174) and the mask is recomputed."""
    from xcp.engine import Stats
    g = torch.Generator(device=gpu).manual_seed(rows)
    y = (torch.randn(rows, C, device=gpu, generator=g) * 2 + 0.7).to(dt)
    gamma = (torch.rand(C, device=gpu, generator=g) + 0.5).requires_grad_(True)
    beta = (torch.randn(C, device=gpu, generator=g) * 0.1).requires_grad_(True)
    rm, rv = torch.zeros(C, device=gpu), torch.ones(C, device=gpu)
    part, R = ops.row_stats(y, rows, C)
    st = Stats(C, gpu)
    bn = {"weight": gamma, "bias": beta, "running_mean": rm, "running_var": rv, "eps": 1e-5, "momentum": 0.1,
          "track": True}
    ops.finalize_stats(part, R, C, rows, bn, True, st)
    yr = y.float().requires_grad_(True)
    rm2, rv2 = torch.zeros(C, device=gpu), torch.ones(C, device=gpu)
    z = F.batch_norm(yr, rm2, rv2, gamma, beta, True, 0.1, 1e-5)
    torch.testing.assert_close(rm, rm2, rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(rv, rv2, rtol=1e-5, atol=1e-6)
    zk = torch.empty(rows, C, device=gpu, dtype=dt)
    ops.bn_act(y, zk, st.scale, st.shift, False, rows, C)
    assert rel_err(zk.float(), z) < (1e-6 if dt == torch.float32 else 1e-2)
    dz = torch.randn(rows, C, device=gpu, generator=g).to(dt)
    (F.relu(z) if relu else z).backward(dz.float())
    dY = torch.empty(rows, C, device=gpu, dtype=dt)
    dg, db = torch.empty(C, device=gpu), torch.empty(C, device=gpu)
    ops.bn_backward(dz, y, rows, C, bn, st, dY, dg, db, relu=relu)
    assert rel_err(dY.float(), yr.grad) < (1e-4 if dt == torch.float32 else 2e-2)
    torch.testing.assert_close(dg, gamma.grad, rtol=1e-4, atol=1e-3)
    torch.testing.assert_close(db, beta.grad, rtol=1e-4, atol=1e-3)


@pytest.mark.parametrize("dt", DTYPES)
def test_bn_padded_channel_pitch(ops, gpu, dt):
    """The 728-channel flow at its 736 pitch: statistics, running buffers and backward over
    the padded rows equal the dense ones on the 728 real channels, and the padding channels get
    zero scale / shift / backward coefficients (so they stay zero downstream)."""
    from xcp.engine import Stats
    rows, C, CP = 3 * 361, 728, 736
    g = torch.Generator(device=gpu).manual_seed(7)
    y = (torch.randn(rows, C, device=gpu, generator=g) * 2 + 0.7).to(dt)
    dz = torch.randn(rows, C, device=gpu, generator=g).to(dt)
    yp, dzp = torch.zeros(rows, CP, device=gpu, dtype=dt), torch.zeros(rows, CP, device=gpu, dtype=dt)
    yp[:, :C], dzp[:, :C] = y, dz
    gamma, beta = torch.rand(C, device=gpu, generator=g) + 0.5, torch.randn(C, device=gpu, generator=g) * 0.1
    res = []
    for (yy, dd, cp) in ((y, dz, C), (yp, dzp, CP)):
        rm, rv = torch.zeros(C, device=gpu), torch.ones(C, device=gpu)
        bn = {"weight": gamma, "bias": beta, "running_mean": rm, "running_var": rv, "eps": 1e-5, "momentum": 0.1,
              "track": True}
        part, R = ops.row_stats(yy, rows, cp)
        st = Stats(cp, gpu)
        ops.finalize_stats(part, R, C, rows, bn, True, st, cp)
        dY = torch.full((rows, cp), float("nan"), device=gpu, dtype=dt)
        dg, db = torch.empty(C, device=gpu), torch.empty(C, device=gpu)
        coef = ops.bn_backward_coef(dd, yy, rows, C, bn, st, dg, db, CP=cp)
        ops.bn_apply_coef(dd, yy, dY, coef, st, rows, cp)
        res.append((st, rm, rv, dY, dg, db, coef))
    (s0, rm0, rv0, d0, g0, b0, _), (s1, rm1, rv1, d1, g1, b1, c1) = res
    for k in ("mean", "invstd", "scale", "shift"):
        torch.testing.assert_close(s1[k][:C], s0[k], rtol=1e-6, atol=1e-6)
        assert torch.all(s1[k][C:] == 0), k
    torch.testing.assert_close(rm1, rm0, rtol=1e-6, atol=1e-7)
    torch.testing.assert_close(rv1, rv0, rtol=1e-6, atol=1e-7)
    assert torch.all(c1.view(3, CP)[:, C:] == 0)
    assert torch.all(d1[:, C:] == 0)
    assert rel_err(d1[:, :C].float(), d0.float()) < 1e-5
    torch.testing.assert_close(g1, g0, rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(b1, b0, rtol=1e-5, atol=1e-5)


@pytest.mark.parametrize("rows,C,CP,relu", [(256 * 147 * 147 // 64, 32, 32, True), (3 * 361, 728, 736, False),
                                             (5, 64, 64, True)])
def test_bn_bwd_finalize_narrow(ops, gpu, rows, C, CP, relu):
    """XCP_FIN_NARROW (the stem BN1 finalize beside conv2's weight gradient): 4-wave workgroups reduce the
    partial rows in another order than the 16-wave form -- the coefficients and the accumulated affine
    gradients agree to fp64 rounding (rtol 1e-6), the padding channels stay zero."""
    from xcp.engine import Stats
    g = torch.Generator(device=gpu).manual_seed(rows + C)
    y = torch.zeros(rows, CP, device=gpu, dtype=torch.bfloat16)
    dz = torch.zeros(rows, CP, device=gpu, dtype=torch.bfloat16)
    y[:, :C] = (torch.randn(rows, C, device=gpu, generator=g) * 2 + 0.7).bfloat16()
    dz[:, :C] = torch.randn(rows, C, device=gpu, generator=g).bfloat16()
    gamma, beta = torch.rand(C, device=gpu, generator=g) + 0.5, torch.randn(C, device=gpu, generator=g) * 0.1
    bn = {"weight": gamma, "bias": beta, "running_mean": torch.zeros(C, device=gpu),
          "running_var": torch.ones(C, device=gpu), "eps": 1e-5, "momentum": 0.1, "track": True}
    part, R = ops.row_stats(y, rows, CP)
    st = Stats(CP, gpu)
    ops.finalize_stats(part, R, C, rows, bn, True, st, CP)
    res = []
    for narrow in (False, True):
        dg, db = torch.ones(C, device=gpu), torch.ones(C, device=gpu)
        coef = ops.bn_backward_coef(dz, y, rows, C, bn, st, dg, db, relu=relu, accumulate=True, CP=CP, narrow=narrow)
        res.append((coef, dg, db))
    torch.cuda.synchronize()
    for a, b in zip(res[0], res[1]):
        torch.testing.assert_close(b, a, rtol=1e-6, atol=1e-7)
    assert torch.all(res[1][0].view(3, CP)[:, C:] == 0)


@pytest.mark.parametrize("dt", DTYPES)
@pytest.mark.parametrize("H", [147, 37, 19, 20])
def test_tail_maxpool_fwd_bwd(ops, gpu, dt, H):
    N, C = 2, 128
    g = torch.Generator(device=gpu).manual_seed(H)
    y = torch.randn(N, C, H, H, device=gpu, generator=g).to(dt)
    s1 = torch.rand(C, device=gpu, generator=g) + 0.5
    t1 = torch.randn(C, device=gpu, generator=g)
    OH = (H - 1) // 2 + 1
    ys = torch.randn(N, C, OH, OH, device=gpu, generator=g).to(dt)
    s2 = torch.rand(C, device=gpu, generator=g) + 0.5
    t2 = torch.randn(C, device=gpu, generator=g)
    zr = (y.float() * s1.view(1, C, 1, 1) + t1.view(1, C, 1, 1)).requires_grad_(True)
    pooled = F.max_pool2d(zr, 3, 2, 1)
    ref = pooled + ys.float() * s2.view(1, C, 1, 1) + t2.view(1, C, 1, 1)
    out = torch.empty(N * OH * OH, C, device=gpu, dtype=dt)
    amax = torch.empty(N * OH * OH * C, device=gpu, dtype=torch.uint8)
    ops.tail_fwd(nhwc(y), s1, t1, True, nhwc(ys), s2, t2, out, amax, N, H, H, C)
    assert rel_err(nchw(out.view(N, OH, OH, C)).float(), ref) < (1e-6 if dt == torch.float32 else 1e-2)
    d = torch.randn(ref.shape, device=gpu, generator=g).to(dt)
    pooled.backward(d.float())
    dz = torch.empty(N * H * H, C, device=gpu, dtype=dt)
    ops.maxpool_bwd(nhwc(d), amax, dz, N, H, H, C)
    assert rel_err(nchw(dz.view(N, H, H, C)).float(), zr.grad) < (1e-6 if dt == torch.float32 else 1e-2)
    from xcp.engine import Stats
    st = Stats(C, gpu)
    st.mean.copy_(torch.randn(C, device=gpu, generator=g))
    st.invstd.copy_(torch.rand(C, device=gpu, generator=g) + 0.5)
    bn = {"weight": s1, "bias": t1, "running_mean": None, "running_var": None, "eps": 1e-5, "momentum": 0.1,
          "track": False}
    rows = N * H * H
    outs = []
    dY = torch.empty(rows, C, device=gpu, dtype=dt)
    dg, db = torch.empty(C, device=gpu), torch.empty(C, device=gpu)
    ops.bn_backward(dz, nhwc(y), rows, C, bn, st, dY, dg, db)
    outs.append((dY, dg, db))
    # accumulate form of the BN affine gradients
    dg2, db2 = dg + 1, db - 2
    ops.bn_backward(dz, nhwc(y), rows, C, bn, st, torch.empty_like(dY), dg2, db2, accumulate=True)
    torch.testing.assert_close(dg2, 2 * dg + 1, rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(db2, 2 * db - 2, rtol=1e-5, atol=1e-5)
    # max-pool backward fused with the BN reduce: same dz bit for bit, same BN backward up to
    # the fp32 summation order of the partials
    dz3 = torch.full_like(dz, float("nan"))
    part, R = ops.maxpool_bwd_bnred(nhwc(d), amax, dz3, nhwc(y), st, N, H, H, C)
    assert torch.equal(dz3, dz)
    dY = torch.empty(rows, C, device=gpu, dtype=dt)
    dg, db = torch.empty(C, device=gpu), torch.empty(C, device=gpu)
    ops.bn_backward(dz3, nhwc(y), rows, C, bn, st, dY, dg, db, part=part, R=R)
    torch.testing.assert_close(dg, outs[0][1], rtol=1e-4, atol=1e-4)
    torch.testing.assert_close(db, outs[0][2], rtol=1e-4, atol=1e-4)
    assert rel_err(dY.float(), outs[0][0].float()) < (1e-5 if dt == torch.float32 else 1e-2)


@pytest.mark.parametrize("dt", DTYPES)
def test_avgpool(ops, gpu, dt):
    N, C, H = 3, 2048, 10
    y = torch.randn(N, C, H, H, device=gpu).to(dt)
    s = torch.rand(C, device=gpu) + 0.5
    t = torch.randn(C, device=gpu)
    zr = (y.float() * s.view(1, C, 1, 1) + t.view(1, C, 1, 1)).requires_grad_(True)
    ref = F.adaptive_avg_pool2d(F.relu(zr), 1).view(N, C)
    Fo = torch.empty(N, C, device=gpu)
    ops.avgpool_fwd(nhwc(y), s, t, Fo, N, H * H, C)
    torch.testing.assert_close(Fo, ref, **tol(dt))
    dF = torch.randn(N, C, device=gpu)
    ref.backward(dF)
    dz = torch.empty(N * H * H, C, device=gpu, dtype=dt)
    ops.avgpool_bwd(dF, nhwc(y), s, t, dz, N, H * H, C)
    assert rel_err(nchw(dz.view(N, H, H, C)).float(), zr.grad) < (1e-6 if dt == torch.float32 else 1e-2)


@pytest.mark.parametrize("dt", DTYPES)
@pytest.mark.parametrize("IH,IW", [(75, 75), (299, 299), (7, 1501), (33, 320), (9, 331)],
                         ids=["75", "299", "wide-perpixel", "row-widest", "tile-331"])
def test_conv1_fwd_wgrad(ops, gpu, dt, IH, IW):
    """Stem conv1 3x3 s2: the row kernels (bf16, frames <= 320 wide), the tiled kernels (fp32 / wider
    frames) and the per-pixel kernels frames wider than the tiles' 64 KB LDS budget fall back to."""
    N = 2
    x = torch.rand(N, 3, IH, IW, device=gpu)
    w = (torch.randn(32, 3, 3, 3, device=gpu) / 5).requires_grad_(True)
    ref = F.conv2d(x, w, None, 2, 0)
    OH, OW = ref.shape[2:]
    Y = torch.empty(N * OH * OW, 32, device=gpu, dtype=dt)
    ops.conv1_fwd(x, w.detach().contiguous(), Y, N, IH, IW)
    assert rel_err(nchw(Y.view(N, OH, OW, 32)).float(), ref) < (1e-6 if dt == torch.float32 else 1e-2)
    dy = torch.randn(ref.shape, device=gpu).to(dt)
    ref.backward(dy.float())
    dW = torch.empty(32 * 27, device=gpu)
    ops.conv1_wgrad(x, nhwc(dy), dW, N, IH, IW)
    torch.cuda.synchronize()
    assert rel_err(dW.view(32, 3, 3, 3), w.grad) < (1e-5 if dt == torch.float32 else 1e-2)


@pytest.mark.parametrize("N,IH,IW", [(3, 299, 299), (2, 65, 64), (5, 17, 23), (1, 31, 320)])
def test_conv1_fwd_stats(ops, gpu, N, IH, IW):
    """conv1 forward with BN1's partial sums: the output equals the plain forward's bit for bit, and
    the partial rows sum to the per-channel sum / sum of squares of the stored output."""
    OH, OW = (IH - 3) // 2 + 1, (IW - 3) // 2 + 1
    g = torch.Generator(device=gpu).manual_seed(7 * N + IW)
    x = torch.rand(N, 3, IH, IW, device=gpu, generator=g)
    w = torch.randn(32, 3, 3, 3, device=gpu, generator=g) / 5
    Y0 = torch.empty(N * OH * OW, 32, device=gpu, dtype=torch.bfloat16)
    Y1 = torch.full_like(Y0, float("nan"))
    ops.conv1_fwd(x, w, Y0, N, IH, IW)
    part, R = ops.conv1_fwd_stats(x, w, Y1, N, IH, IW)
    torch.cuda.synchronize()
    assert torch.equal(Y0, Y1)
    sums = part.view(R, 2, 32).double().sum(0)
    yd = Y1.double()
    torch.testing.assert_close(sums[0], yd.sum(0), rtol=1e-5, atol=1e-3)
    torch.testing.assert_close(sums[1], (yd * yd).sum(0), rtol=1e-5, atol=1e-3)
    ref = F.conv2d(x, w, None, 2, 0)
    assert rel_err(nchw(Y1.view(N, OH, OW, 32)).float(), ref) < 4e-3   # the bf16 output rounding alone


@pytest.mark.parametrize("N,IH,IW", [(3, 299, 299), (2, 65, 64), (5, 17, 23), (1, 31, 320)])
@pytest.mark.parametrize("relu", [True, False])
def test_conv1_wgrad_bn_fused(ops, gpu, N, IH, IW, relu):
    """conv1's weight gradient with BN1's backward apply formed on load (xcp_conv1_wgrad_bn) equals the
    apply kernel's stored dC1 fed to xcp_conv1_wgrad bit for bit (same bf16 rounding, same summation
    order), and the fp32 conv2d weight gradient of that dC1."""
    assert ops.conv1_wgrad_fused(torch.bfloat16, IH, IW)
    OH, OW = (IH - 3) // 2 + 1, (IW - 3) // 2 + 1
    rows, C = N * OH * OW, 32
    g = torch.Generator(device=gpu).manual_seed(N * IH + IW)
    x = torch.rand(N, 3, IH, IW, device=gpu, generator=g)
    dZ = torch.randn(rows, C, device=gpu, generator=g).bfloat16()
    Y = torch.randn(rows, C, device=gpu, generator=g).bfloat16()
    coef = torch.randn(3 * C, device=gpu, generator=g)
    st = {"scale": torch.randn(C, device=gpu, generator=g), "shift": torch.randn(C, device=gpu, generator=g) * 0.3}
    dC1 = torch.empty(rows, C, device=gpu, dtype=torch.bfloat16)
    ops.bn_apply_coef(dZ, Y, dC1, coef, st, rows, C, relu=relu)
    ref = torch.empty(32 * 27, device=gpu)
    ops.conv1_wgrad(x, dC1, ref, N, IH, IW)
    out = torch.full((32 * 27,), float("nan"), device=gpu)
    ops.conv1_wgrad_bn(x, dZ, Y, coef, st, out, N, IH, IW, C, relu=relu)
    acc = torch.ones(32 * 27, device=gpu)
    ops.conv1_wgrad_bn(x, dZ, Y, coef, st, acc, N, IH, IW, C, relu=relu, accumulate=True)
    torch.cuda.synchronize()
    assert torch.equal(out, ref)
    torch.testing.assert_close(acc, ref + 1, rtol=1e-6, atol=1e-5)
    # (the matrix-core products split each input into a bf16 head and tail: exact to ~2^-17)
    w = torch.zeros(32, 3, 3, 3, device=gpu, requires_grad=True)
    F.conv2d(x, w, None, 2, 0).backward(nchw(dC1.view(N, OH, OW, C)).float())
    assert rel_err(out.view(32, 3, 3, 3), w.grad) < 2e-5


def test_permute3(ops, gpu):
    x = torch.randn(5, 7, 9, device=gpu)
    for perm in [(0, 1, 2), (0, 2, 1), (1, 0, 2), (1, 2, 0), (2, 0, 1), (2, 1, 0)]:
        out = torch.empty(x.numel(), device=gpu)
        ops.permute3(x, out, 5, 7, 9, perm)
        assert torch.equal(out.view([x.shape[p] for p in perm]), x.permute(*perm))
    ob = torch.empty(x.numel(), device=gpu, dtype=torch.bfloat16)
    ops.permute3(x, ob, 5, 7, 9, (2, 0, 1))
    assert torch.equal(ob.view(9, 5, 7), x.permute(2, 0, 1).to(torch.bfloat16))


@pytest.mark.parametrize("kernel", ["register", "generic"])
@pytest.mark.parametrize("H,T", [(128, 16), (512, 12)])
def test_lstm_module_vs_oracle(ops, gpu, golden, H, T, kernel):
    """Both recurrence kernel families (LSTM.xcp_kernel 0: register-resident / per-step, 1:
    generic) against the reference nn.LSTM goldens."""
    import numpy as np
    from xcp.lstm import LSTM
    g = golden("lstm.npz")
    torch.manual_seed(0)
    lstm = LSTM(2048, H, 1, batch_first=True).to(gpu)
    lstm.xcp_kernel = 0 if kernel == "register" else 1
    x = torch.randn((2, T, 2048), generator=torch.Generator().manual_seed(555)).to(gpu).requires_grad_(True)
    o, (h, c) = lstm(x)
    p = f"H{H}"
    np.testing.assert_allclose(o.detach().cpu().numpy(), g[f"{p}/out"], rtol=1e-4, atol=1e-5)
    np.testing.assert_allclose(h.detach().cpu().numpy(), g[f"{p}/h_n"], rtol=1e-4, atol=1e-5)
    np.testing.assert_allclose(c.detach().cpu().numpy(), g[f"{p}/c_n"], rtol=1e-4, atol=1e-5)
    r = torch.randn(o.shape, generator=torch.Generator().manual_seed(556)).to(gpu)
    rh = torch.randn(h.shape, generator=torch.Generator().manual_seed(557)).to(gpu)
    ((o * r).sum() + (c * rh).sum()).backward()
    np.testing.assert_allclose(x.grad.cpu().numpy(), g[f"{p}/dx"], rtol=1e-3, atol=1e-5)
    for n, prm in lstm.named_parameters():
        ref = g[f"{p}/grad/{n}"]
        if ref.ndim == 0:
            np.testing.assert_allclose(prm.grad.double().norm().item(), ref, rtol=1e-4)
        else:
            np.testing.assert_allclose(prm.grad.cpu().numpy(), ref, rtol=1e-3, atol=1e-5)


@pytest.mark.parametrize("kernel", ["persistent", "step", "generic"])
def test_lstm_t120_vs_reference(ops, gpu, golden, monkeypatch, kernel):
    """XceptionLSTMA's own recurrence -- nn.LSTM(2048, 512) over T = 120 MFCC frames
    (XceptionLSTMA.py:14-19, audio_dataloader.py:20,39) -- through the three kernel families H = 512
    can take (persistent: XCP_LSTM_PERSIST=1, one launch each way -- the default runs the forward
    that way and the backward per step; step: XCP_LSTM_PERSIST=0, 120 launches each way carrying h
    and c; generic) against the reference's own values (lstm_t120.npz): out /
    h_n / c_n at 1e-4, every time step's output norm at 1e-4 (the error must not grow over the 120
    steps), dx and the parameter gradients at 1e-3."""
    import numpy as np
    from xcp.lstm import LSTM
    g = golden("lstm_t120.npz")
    B, T, H = int(g["B"]), int(g["T"]), int(g["H"])
    monkeypatch.setenv("XCP_LSTM_PERSIST", "0" if kernel == "step" else "1")
    torch.manual_seed(0)
    lstm = LSTM(2048, H, 1, batch_first=True).to(gpu)
    lstm.xcp_kernel = 1 if kernel == "generic" else 0
    x = torch.randn((B, T, 2048), generator=torch.Generator().manual_seed(555)).to(gpu).requires_grad_(True)
    o, (h, c) = lstm(x)
    oc = o.detach().double().cpu()
    np.testing.assert_allclose(oc.reshape(-1).numpy()[g["out/idx"]], g["out/val"], rtol=1e-4, atol=1e-5)
    np.testing.assert_allclose(oc.norm(dim=2).numpy(), g["out_step_norm"], rtol=1e-4)
    np.testing.assert_allclose(o.detach()[:, -1].cpu().numpy(), g["out_last"], rtol=1e-4, atol=1e-5)
    np.testing.assert_allclose(h.detach().cpu().numpy(), g["h_n"], rtol=1e-4, atol=1e-5)
    np.testing.assert_allclose(c.detach().cpu().numpy(), g["c_n"], rtol=1e-4, atol=1e-5)
    r = torch.randn(o.shape, generator=torch.Generator().manual_seed(556)).to(gpu)
    rc = torch.randn(c.shape, generator=torch.Generator().manual_seed(557)).to(gpu)
    ((o * r).sum() + (c * rc).sum()).backward()
    dx = x.grad.double().cpu()
    np.testing.assert_allclose(dx.reshape(-1).numpy()[g["dx/idx"]], g["dx/val"], rtol=1e-3, atol=1e-5)
    np.testing.assert_allclose(dx.norm(dim=2).numpy(), g["dx_step_norm"], rtol=1e-3)
    for n, prm in lstm.named_parameters():
        gr = prm.grad.double().cpu()
        np.testing.assert_allclose(gr.norm().item(), g[f"gradnorm/{n}"], rtol=1e-3, err_msg=n)
        np.testing.assert_allclose(gr.reshape(-1).numpy()[g[f"grad/{n}/idx"]], g[f"grad/{n}/val"], rtol=1e-3,
                                   atol=1e-5, err_msg=n)
        if f"gradfull/{n}" in g:
            np.testing.assert_allclose(gr.numpy(), g[f"gradfull/{n}"], rtol=1e-3, atol=1e-5, err_msg=n)
    assert ops.lstm_sync_error() == 0


@pytest.mark.parametrize("B,T,H", [(16, 120, 512), (20, 37, 512), (3, 5, 256), (32, 9, 256)])
def test_lstm_persistent_vs_step_kernels(ops, gpu, monkeypatch, B, T, H):
    """The persistent recurrence (one launch per direction, W_hh in VGPRs, step hand-off through
    sharded counters) against the per-step kernels on the same inputs, with every optional operand
    (dout, dh_n, dc_n): outputs, states, gates and the pre-activation gradients within 1e-5 relative
    (only the summation order of the W_hh dot products differs).  B = 20 / 32 take the second
    clip pass, B = 3 a partial clip group; no launch may report a poll timeout."""
    G4 = 4 * H
    gen = torch.Generator(device=gpu).manual_seed(B * 1000 + T + H)
    xp = torch.randn(B, T, G4, device=gpu, generator=gen)
    whh = torch.randn(G4, H, device=gpu, generator=gen) / H ** 0.5
    bih, bhh = torch.randn(G4, device=gpu, generator=gen) * 0.1, torch.randn(G4, device=gpu, generator=gen) * 0.1
    dout = torch.randn(B, T, H, device=gpu, generator=gen)
    dhn, dcn = torch.randn(B, H, device=gpu, generator=gen), torch.randn(B, H, device=gpu, generator=gen)
    res = {}
    for form in ("0", "1"):
        monkeypatch.setenv("XCP_LSTM_PERSIST", form)
        f = {k: torch.full((B, T, n), float("nan"), device=gpu) for k, n in
             (("out", H), ("hprev", H), ("cst", H), ("gates", G4))}
        hn, cn = torch.empty(B, H, device=gpu), torch.empty(B, H, device=gpu)
        ops.lstm_fwd(xp, whh, None, bih, bhh, f["out"], f["hprev"], f["cst"], f["gates"], hn, cn, B, T, H)
        dg = torch.full((B, T, G4), float("nan"), device=gpu)
        ops.lstm_bwd(dout, dhn, dcn, whh, f["cst"], f["gates"], dg, B, T, H)
        torch.cuda.synchronize()
        res[form] = dict(f, hn=hn, cn=cn, dg=dg)
    assert ops.lstm_sync_error() == 0
    for k, want in res["0"].items():
        got = res["1"][k]
        assert not torch.isnan(got).any(), k
        err = ((got - want).norm() / want.norm()).item()
        assert err < 1e-5, (k, err)


@pytest.mark.parametrize("cg", ["cg", "cg2"])
@pytest.mark.parametrize("B,T,H", [(16, 9, 512), (3, 5, 256), (13, 7, 512)])
def test_lstm_bwd_clip_grouped_bitwise(ops, gpu, monkeypatch, B, T, H, cg):
    """XCP_LSTM_BWD=cg / cg2 (the persistent backward split by clips as well as units, one / two clips per wave) against
    the gather form it restates: the same per-lane chains and reduction tree, so dgates bit for bit; every
    optional operand; B = 13 leaves idle waves in the last clip group; no poll timeout."""
    G4 = 4 * H
    gen = torch.Generator(device=gpu).manual_seed(B * 100 + T + H)
    xp = torch.randn(B, T, G4, device=gpu, generator=gen)
    whh = torch.randn(G4, H, device=gpu, generator=gen) / H ** 0.5
    bih, bhh = torch.zeros(G4, device=gpu), torch.zeros(G4, device=gpu)
    dout = torch.randn(B, T, H, device=gpu, generator=gen)
    dhn, dcn = torch.randn(B, H, device=gpu, generator=gen), torch.randn(B, H, device=gpu, generator=gen)
    monkeypatch.setenv("XCP_LSTM_PERSIST", "1")
    f = {k: torch.empty(B, T, n, device=gpu) for k, n in (("out", H), ("hprev", H), ("cst", H), ("gates", G4))}
    hn, cn = torch.empty(B, H, device=gpu), torch.empty(B, H, device=gpu)
    ops.lstm_fwd(xp, whh, None, bih, bhh, f["out"], f["hprev"], f["cst"], f["gates"], hn, cn, B, T, H)
    res = {}
    for form in ("gather", cg):
        monkeypatch.setenv("XCP_LSTM_BWD", form)
        dg = torch.full((B, T, G4), float("nan"), device=gpu)
        ops.lstm_bwd(dout, dhn, dcn, whh, f["cst"], f["gates"], dg, B, T, H)
        torch.cuda.synchronize()
        res[form] = dg
    assert ops.lstm_sync_error() == 0
    assert not torch.isnan(res[cg]).any()
    assert torch.equal(res[cg], res["gather"])


@pytest.mark.parametrize("kernel", ["register", "generic"])
def test_lstm_h64_vs_oracle(ops, gpu, kernel):
    """H = 64 (the second register-resident instantiation) against the oracle's nn.LSTM
    restatement (oracle/xception_oracle.py lstm_forward, autograd for the gradients)."""
    from oracle import xception_oracle as O
    from xcp.lstm import LSTM
    torch.manual_seed(3)
    lstm = LSTM(256, 64, 1, batch_first=True).to(gpu)
    lstm.xcp_kernel = 0 if kernel == "register" else 1
    x = torch.randn((3, 9, 256), generator=torch.Generator().manual_seed(7))
    xg = x.to(gpu).requires_grad_(True)
    o, (h, c) = lstm(xg)
    r = torch.randn(o.shape, generator=torch.Generator().manual_seed(8))
    (o * r.to(gpu)).sum().backward()
    cp = {n: p.detach().cpu().clone().requires_grad_(True) for n, p in lstm.named_parameters()}
    xc = x.clone().requires_grad_(True)
    ro, rh, rc = O.lstm_forward(xc, cp["weight_ih_l0"], cp["weight_hh_l0"], cp["bias_ih_l0"], cp["bias_hh_l0"])
    (ro * r).sum().backward()
    torch.testing.assert_close(o.detach().cpu(), ro.detach(), rtol=1e-4, atol=1e-5)
    torch.testing.assert_close(c.detach().cpu(), rc.detach(), rtol=1e-4, atol=1e-5)
    torch.testing.assert_close(xg.grad.cpu(), xc.grad, rtol=1e-3, atol=1e-5)
    for n, p in lstm.named_parameters():
        torch.testing.assert_close(p.grad.cpu(), cp[n].grad, rtol=1e-3, atol=1e-5)


@pytest.mark.parametrize("H,B,T", [(256, 5, 7), (512, 17, 4), (1024, 3, 3), (512, 32, 3), (1024, 20, 2)])
def test_lstm_step_kernels_vs_oracle(ops, gpu, H, B, T):
    """Per-step recurrence kernels (large H: one launch per time step over H/2 workgroups)
    against the oracle's nn.LSTM restatement, including a carried-in gradient on c_n.  The
    last two batches exceed the per-step kernels' LDS budget, so they run the generic kernels
    (the forward must build the transposed W_hh those read)."""
    from oracle import xception_oracle as O
    from xcp.lstm import LSTM
    torch.manual_seed(H)
    lstm = LSTM(128, H, 1, batch_first=True).to(gpu)
    x = torch.randn((B, T, 128), generator=torch.Generator().manual_seed(H + 1))
    xg = x.to(gpu).requires_grad_(True)
    o, (h, c) = lstm(xg)
    r = torch.randn(o.shape, generator=torch.Generator().manual_seed(H + 2))
    rc = torch.randn(c.shape, generator=torch.Generator().manual_seed(H + 3))
    ((o * r.to(gpu)).sum() + (c * rc.to(gpu)).sum()).backward()
    cp = {n: p.detach().cpu().clone().requires_grad_(True) for n, p in lstm.named_parameters()}
    xc = x.clone().requires_grad_(True)
    ro, rh, rcn = O.lstm_forward(xc, cp["weight_ih_l0"], cp["weight_hh_l0"], cp["bias_ih_l0"], cp["bias_hh_l0"])
    ((ro * r).sum() + (rcn * rc).sum()).backward()
    torch.testing.assert_close(o.detach().cpu(), ro.detach(), rtol=1e-4, atol=1e-5)
    torch.testing.assert_close(h.detach().cpu(), rh.detach(), rtol=1e-4, atol=1e-5)
    torch.testing.assert_close(c.detach().cpu(), rcn.detach(), rtol=1e-4, atol=1e-5)
    torch.testing.assert_close(xg.grad.cpu(), xc.grad, rtol=1e-3, atol=1e-5)
    for n, p in lstm.named_parameters():
        torch.testing.assert_close(p.grad.cpu(), cp[n].grad, rtol=1e-3, atol=1e-5)


@pytest.mark.parametrize("N,IH,IW", [(2, 149, 149), (3, 21, 38), (1, 6, 147)])
def test_conv3x3_stem_fwd_dgrad(ops, gpu, N, IH, IW):
    """Direct MFMA stem conv2 (conv3.hip) against F.conv2d / its input gradient (bf16
    operands, fp32 reference on the same rounded values), BN partial sums against the
    stored output; the 149 case is the 299^2 bench shape."""
    g = torch.Generator(device=gpu).manual_seed(IH * IW)
    x = torch.randn(N, 32, IH, IW, device=gpu, generator=g).bfloat16()
    w = (torch.randn(64, 32, 3, 3, device=gpu, generator=g) / 288 ** 0.5).bfloat16()
    OH, OW = IH - 2, IW - 2
    R = ops.conv3x3_parts(0, N, IH, IW)
    stats = torch.full((R, 2, 64), float("nan"), device=gpu)
    Y = torch.full((N * OH * OW, 64), float("nan"), device=gpu, dtype=torch.bfloat16)
    Wp = w.permute(0, 2, 3, 1).reshape(64, 9 * 32).contiguous()          # [co][tap][ci]
    ops.conv3x3(0, nhwc(x), Wp, Y, stats, N, IH, IW)
    ref = F.conv2d(x.float(), w.float())
    assert rel_err(nchw(Y.view(N, OH, OW, 64)).float(), ref) < 1e-2
    s, Yd = stats.double().sum(0), Y.double()
    torch.testing.assert_close(s[0], Yd.sum(0), rtol=1e-5, atol=1e-3)
    torch.testing.assert_close(s[1], (Yd * Yd).sum(0), rtol=1e-5, atol=1e-3)
    # input gradient: a 64 -> 32 conv of the pad-2 gradient with the flipped kernel
    dy = torch.randn(N, 64, OH, OW, device=gpu, generator=g).bfloat16()
    WT = w.permute(1, 2, 3, 0).reshape(32, 9 * 64).contiguous()          # [ci][tap][co]
    DX = torch.full((N * IH * IW, 32), float("nan"), device=gpu, dtype=torch.bfloat16)
    ops.conv3x3(1, nhwc(dy), WT, DX, None, N, OH, OW)
    ref_dx = torch.nn.grad.conv2d_input((N, 32, IH, IW), w.float(), dy.float())
    assert rel_err(nchw(DX.view(N, IH, IW, 32)).float(), ref_dx) < 1e-2
    # weight gradient (slabs + colreduce) against conv2d_weight on the same bf16 operands
    dW = torch.full((64 * 288,), float("nan"), device=gpu)
    ops.conv3x3_wgrad(nhwc(dy), nhwc(x), dW, N, IH, IW)
    ref_dw = torch.nn.grad.conv2d_weight(x.float(), (64, 32, 3, 3), dy.float())
    got = dW.view(64, 3, 3, 32).permute(0, 3, 1, 2)
    assert rel_err(got, ref_dw) < 1e-4


@pytest.mark.parametrize("form", ["0", "1", "2"])
@pytest.mark.parametrize("N,IH,IW", [(2, 149, 149), (3, 21, 38), (1, 6, 147), (2, 12, 160), (3, 3, 3), (1, 40, 34)])
def test_conv3x3_wgrad_forms(ops, gpu, monkeypatch, form, N, IH, IW):
    """The stem conv2 weight gradient in its three forms (XCP_CONV3_WGRAD: 0 = one dY and nine shifted X
    fragments per chunk, 1 = the reduction indexed by input pixel -- three X and three shifted dY fragments,
    2 = the same with two co blocks per wave and the chunk halves summed through LDS) against conv2d_weight
    on the same bf16 operands, plain and with BN1 + ReLU applied on load (bitwise against the activated
    input within each form); widths up to 160 (the shifted forms' ring), single-row and single-column images."""
    monkeypatch.setenv("XCP_CONV3_WGRAD", form)
    g = torch.Generator(device=gpu).manual_seed(IH * 3 + IW)
    rows = N * IH * IW
    x = (torch.randn(rows, 32, device=gpu, generator=g) * 1.5 + 0.3).bfloat16()
    sc = torch.rand(32, device=gpu, generator=g) + 0.4
    sh = torch.randn(32, device=gpu, generator=g) * 0.5
    a = torch.empty_like(x)
    ops.bn_act(x, a, sc, sh, True, rows, 32)
    OH, OW = IH - 2, IW - 2
    dy = torch.randn(N * OH * OW, 64, device=gpu, generator=g).bfloat16()
    assert ops.conv3x3_wgrad_parts(N, IH, IW) > 0
    dws = []
    for src, kw in ((a, {}), (x, {"in_scale": sc, "in_shift": sh})):
        dW = torch.full((64 * 288,), float("nan"), device=gpu)
        ops.conv3x3_wgrad(dy, src, dW, N, IH, IW, **kw)
        dws.append(dW)
    torch.cuda.synchronize()
    assert torch.equal(dws[0], dws[1])
    ref_dw = torch.nn.grad.conv2d_weight(nchw(a.view(N, IH, IW, 32)).float(), (64, 32, 3, 3),
                                         nchw(dy.view(N, OH, OW, 64)).float())
    assert rel_err(dws[0].view(64, 3, 3, 32).permute(0, 3, 1, 2), ref_dw) < 1e-4


@pytest.mark.parametrize("N,IH,IW", [(2, 149, 149), (3, 21, 38), (1, 6, 147)])
def test_conv3x3_bn_relu_on_load_bitwise(ops, gpu, N, IH, IW):
    """in_scale / in_shift (the stem's BN1 + ReLU applied to each staged conv1-output tile, forward and
    weight gradient) against bn_act into a separate activation followed by the plain kernels: the same
    rounded activations meet the same MFMAs, so the outputs, the BN partial sums and the weight-gradient
    slabs are bitwise equal (junk activated past the image only meets rows / columns never stored or a
    zero dY)."""
    g = torch.Generator(device=gpu).manual_seed(IH + 7 * IW)
    rows = N * IH * IW
    x = (torch.randn(rows, 32, device=gpu, generator=g) * 1.5 + 0.3).bfloat16()
    sc = torch.rand(32, device=gpu, generator=g) + 0.4
    sh = torch.randn(32, device=gpu, generator=g) * 0.5
    Wp = (torch.randn(64, 288, device=gpu, generator=g) / 17).bfloat16()
    a = torch.empty_like(x)
    ops.bn_act(x, a, sc, sh, True, rows, 32)
    OH, OW = IH - 2, IW - 2
    R = ops.conv3x3_parts(0, N, IH, IW)
    outs = []
    for src, kw in ((a, {}), (x, {"in_scale": sc, "in_shift": sh})):
        stats = torch.full((R, 2, 64), float("nan"), device=gpu)
        Y = torch.full((N * OH * OW, 64), float("nan"), device=gpu, dtype=torch.bfloat16)
        ops.conv3x3(0, src, Wp, Y, stats, N, IH, IW, **kw)
        outs.append((Y, stats))
    assert torch.equal(outs[0][0], outs[1][0])
    assert torch.equal(outs[0][1], outs[1][1])
    dy = torch.randn(N * OH * OW, 64, device=gpu, generator=g).bfloat16()
    dws = []
    for src, kw in ((a, {}), (x, {"in_scale": sc, "in_shift": sh})):
        dW = torch.full((64 * 288,), float("nan"), device=gpu)
        ops.conv3x3_wgrad(dy, src, dW, N, IH, IW, **kw)
        dws.append(dW)
    assert torch.equal(dws[0], dws[1])
    ref_dw = torch.nn.grad.conv2d_weight(nchw(a.view(N, IH, IW, 32)).float(), (64, 32, 3, 3),
                                         nchw(dy.view(N, OH, OW, 64)).float())
    assert rel_err(dws[1].view(64, 3, 3, 32).permute(0, 3, 1, 2), ref_dw) < 1e-4


@pytest.mark.parametrize("N,IH,IW", [(3, 149, 149), (2, 9, 40)])
def test_conv3x3_fwd_two_workgroup_form(ops, gpu, monkeypatch, N, IH, IW):
    """XCP_CONV3_FWD_2WG=1 (two 4-wave workgroups per CU on 2-row tiles): the same MFMAs per output
    item, so the output is bitwise the one-workgroup form's; the BN partial rows (one per workgroup)
    sum to the same statistics."""
    g = torch.Generator(device=gpu).manual_seed(IH + N)
    x = torch.randn(N * IH * IW, 32, device=gpu, generator=g).bfloat16()
    Wp = (torch.randn(64, 288, device=gpu, generator=g) / 17).bfloat16()
    OH, OW = IH - 2, IW - 2
    outs = []
    for v in ("0", "1"):
        monkeypatch.setenv("XCP_CONV3_FWD_2WG", v)
        R = ops.conv3x3_parts(0, N, IH, IW)
        stats = torch.full((R, 2, 64), float("nan"), device=gpu)
        Y = torch.full((N * OH * OW, 64), float("nan"), device=gpu, dtype=torch.bfloat16)
        ops.conv3x3(0, x, Wp, Y, stats, N, IH, IW)
        torch.cuda.synchronize()
        outs.append((Y, stats.double().sum(0)))
    assert torch.equal(outs[0][0], outs[1][0])
    torch.testing.assert_close(outs[1][1], outs[0][1], rtol=1e-6, atol=1e-3)


@pytest.mark.parametrize("max_norm", [None, 1.0, 1e-3])
def test_fused_adam_clip_vs_torch(ops, gpu, max_norm):
    """xcp.optim.FusedAdamClip (csrc/optim.hip) against clip_grad_norm_ + torch.optim.Adam (L2
    weight decay) over three steps, on tensors below, at and above the 16384-element chunk."""
    from xcp.optim import FusedAdamClip
    g = torch.Generator(device=gpu).manual_seed(11)
    shapes = [(3,), (128, 129), (16384,), (40000,), (7, 5, 3, 3)]
    a = [torch.randn(s, device=gpu, generator=g).requires_grad_(True) for s in shapes]
    b = [t.detach().clone().requires_grad_(True) for t in a]
    opt_a = FusedAdamClip(a, lr=1e-2, weight_decay=1e-2, max_norm=max_norm)
    opt_b = torch.optim.Adam(b, lr=1e-2, weight_decay=1e-2)
    for step in range(3):
        grads = [torch.randn(s, device=gpu, generator=g) for s in shapes]
        for p, q, gr in zip(a, b, grads):
            p.grad = gr.clone()
            q.grad = gr.clone()
        na = opt_a.step()
        if max_norm is not None:
            nb = torch.nn.utils.clip_grad_norm_(b, max_norm)
            torch.testing.assert_close(na, nb, rtol=1e-5, atol=0)
        else:
            assert na is None
        opt_b.step()
        for p, q in zip(a, b):
            torch.testing.assert_close(p.detach(), q.detach(), rtol=1e-5, atol=1e-6)


def test_fused_adam_clip_load_state_dict_resume(ops, gpu):
    """step -> load_state_dict(torch.optim.Adam's state_dict) -> step against torch.optim.Adam
    with the gradient tensors kept in place (the GradBuckets pattern: param.grad views of one flat
    buffer whose pointers never change), so a chunk table cached before the load would still
    point at the replaced moment buffers (the cache key holds every row pointer and
    load_state_dict drops the tables)."""
    from xcp.optim import FusedAdamClip
    g = torch.Generator(device=gpu).manual_seed(12)
    shapes = [(5,), (64, 33), (20000,)]
    a = [torch.randn(s, device=gpu, generator=g).requires_grad_(True) for s in shapes]
    b = [t.detach().clone().requires_grad_(True) for t in a]
    for p in a + b:
        p.grad = torch.zeros_like(p)
    opt_a = FusedAdamClip(a, lr=1e-2, weight_decay=1e-2, max_norm=1.0)
    opt_b = torch.optim.Adam(b, lr=1e-2, weight_decay=1e-2)

    def step(k):
        for p, q in zip(a, b):
            gr = torch.randn(p.shape, device=gpu, generator=g) * (1.0 + k)
            p.grad.copy_(gr)
            q.grad.copy_(gr)
        opt_a.step()
        torch.nn.utils.clip_grad_norm_(b, 1.0)
        opt_b.step()

    for k in range(2):
        step(k)
    # a different trajectory's state (torch's, after extra steps) replaces both optimisers' state
    for k in range(2, 4):
        for q in b:
            q.grad.copy_(torch.randn(q.shape, device=gpu, generator=g))
        torch.nn.utils.clip_grad_norm_(b, 1.0)
        opt_b.step()
    import copy
    sd = copy.deepcopy(opt_b.state_dict())   # a checkpoint's copy (state_dict() returns the live tensors)
    opt_a.load_state_dict(sd)
    with torch.no_grad():
        for p, q in zip(a, b):
            p.copy_(q)
    for k in range(4, 6):
        step(k)
    for p, q in zip(a, b):
        torch.testing.assert_close(p.detach(), q.detach(), rtol=1e-5, atol=1e-6)
    for p, q in zip(a, b):
        torch.testing.assert_close(opt_a.state[p]["exp_avg"], opt_b.state[q]["exp_avg"], rtol=1e-5, atol=1e-7)


@pytest.mark.parametrize("loop", ["4", "2"])
@pytest.mark.parametrize("M,N,K,ref", [(92416, 736, 736, 2), (5120 * 9, 1024, 736, 2), (2048 * 7 + 256, 512, 64, 2),
                                       (256 * 506 + 77, 256, 200, 2), (256 * 600 + 77, 256, 448, 2),
                                       (256 * 300 + 5, 512, 128, 2)])
def test_gemm_nt_persistent_bitwise(ops, gpu, monkeypatch, M, N, K, ref, loop):
    """The persistent 256x256 kernel (tile 3, every row on it; loop 4: gemm_nt256p_kernel, loop 2:
    gemm_nt256q_kernel's two MFMA phases per K-tile) computes every tile with the one-shot kernel's
    MFMA order: identical output bits against tile 2 (the one-shot kernel for every row), across
    several tiles per workgroup (the prefetch / epilogue overlap must not change a value).  The BN
    statistics are bitwise too for loop 4; loop 2 reduces each 64-row half of a wave's rows over the
    wave and adds the two (its epilogue runs in two halves), so its sums differ by fp32 rounding only
    (1e-6 relative here).  K = 128: two K-tiles per tile, the shortest the two-phase loop runs."""
    monkeypatch.setenv("XCP_NT_LOOP", loop)
    tile = 3
    g = torch.Generator(device=gpu).manual_seed(M + N)
    A = torch.randn(M, K, device=gpu, generator=g).bfloat16()
    B = (torch.randn(N, K, device=gpu, generator=g) / K ** 0.5).bfloat16()
    R = ops.nt_stat_rows(M)
    outs = []
    for t in (ref, tile):
        C = torch.full((M, N), float("nan"), device=gpu, dtype=torch.bfloat16)
        part = torch.full((R, 2, N), float("nan"), device=gpu)
        ops.gemm_nt(A, B, C, M, N, K, stats=part, tile=t)
        outs.append((C, part))
    torch.cuda.synchronize()
    assert torch.equal(outs[0][0], outs[1][0])
    if loop == "4":
        assert torch.equal(outs[0][1], outs[1][1])
    else:
        assert not torch.isnan(outs[1][1]).any()
        torch.testing.assert_close(outs[1][1], outs[0][1], rtol=1e-6, atol=1e-6 * outs[0][1].abs().max().item())


@pytest.mark.parametrize("M,N,K", [(92416, 736, 736), (256 * 600 + 77, 256, 448), (5120 * 9, 1024, 736)])
def test_gemm_nt_persistent_tile_queue_bitwise(ops, gpu, M, N, K):
    """Calls without BN statistics (the backward's input gradients) take the persistent kernel's tiles
    from a per-stream queue (XCP_NT_DYNQ): identical bits against the one-shot kernel, over repeated
    launches (each launch's last fetch resets the counter) and on two streams at once (one counter
    each)."""
    g = torch.Generator(device=gpu).manual_seed(M + 3 * N)
    A = torch.randn(M, K, device=gpu, generator=g).bfloat16()
    B = (torch.randn(N, K, device=gpu, generator=g) / K ** 0.5).bfloat16()
    ref = torch.full((M, N), float("nan"), device=gpu, dtype=torch.bfloat16)
    ops.gemm_nt(A, B, ref, M, N, K, tile=2)
    for _ in range(3):
        C = torch.full((M, N), float("nan"), device=gpu, dtype=torch.bfloat16)
        ops.gemm_nt(A, B, C, M, N, K, tile=3)
        torch.cuda.synchronize()
        assert torch.equal(C, ref)
    s1, s2 = torch.cuda.Stream(gpu), torch.cuda.Stream(gpu)
    outs = []
    for st in (s1, s2, s1, s2):
        st.wait_stream(torch.cuda.current_stream(gpu))
        with torch.cuda.stream(st):
            C = torch.full((M, N), float("nan"), device=gpu, dtype=torch.bfloat16)
            ops.gemm_nt(A, B, C, M, N, K, tile=3)
        outs.append(C)
    torch.cuda.synchronize()
    for C in outs:
        assert torch.equal(C, ref)


def test_reduce_batch_bitwise(ops, gpu):
    """ReduceBatch (xcp_colreduce_multi: up to 16 reductions per launch, two-level jobs split over
    two launches) gives bitwise reduce_slabs' outputs, for one-level and two-level shapes, a slab
    pitch wider than L, the accumulate form, an output off the 16-B grid (reduced on its own),
    and more than 16 jobs."""
    g = torch.Generator(device=gpu).manual_seed(5)
    shapes = [(14, 736 * 736, None), (300, 728 * 9, 736 * 9), (40, 128 * 9, None), (3, 64, None), (129, 256 * 9, None)]
    shapes = shapes * 4   # 20 jobs: two launches per level
    jobs = []
    for i, (S, L, ld) in enumerate(shapes):
        P = torch.randn(S * (ld or L), device=gpu, generator=g)
        o0 = torch.randn(L + 1, device=gpu, generator=g)
        o1 = o0.clone()
        if i % 5 == 4:   # an output view off the 16-B grid (a parameter gradient view of a flat buffer)
            o0, o1 = o0[1:], o1[1:]
        else:
            o0, o1 = o0[:L], o1[:L]
        jobs.append((P, S, L, ld, o0, o1, i % 3 == 0))
    rb = ops.ReduceBatch()
    for P, S, L, ld, o0, o1, acc in jobs:
        ops.reduce_slabs(P, S, L, o0, acc, ld=ld)
        rb.add(P, S, L, o1, acc, ld=ld)
    rb.flush()
    torch.cuda.synchronize()
    for P, S, L, ld, o0, o1, acc in jobs:
        assert torch.equal(o0, o1), (S, L, ld, acc)


def test_permute_batch_plans(ops, gpu):
    """The batched weight pack (xcp_permute3_batch): every job type the engine packs -- row copy
    into a padded pitch, 2-D transpose into a padded pitch, batched transposes (conv2 [co][tap][ci]),
    the (1, 2, 0) transpose (conv2T) -- plus a permutation outside those forms (per-element path),
    in one launch, bf16 and fp32 destinations, against torch.permute (exact: a cast of fp32 values)."""
    g = torch.Generator(device=gpu).manual_seed(3)
    specs = [((728, 728, 1), (0, 1, 2), 736, torch.bfloat16), ((728, 728, 1), (1, 0, 2), 736, torch.bfloat16),
             ((1024, 728, 1), (1, 0, 2), 1024, torch.bfloat16), ((736, 9, 1), (1, 0, 2), 736, torch.float32),
             ((64, 32, 9), (0, 2, 1), None, torch.bfloat16), ((64, 32, 9), (1, 2, 0), None, torch.bfloat16),
             ((5, 7, 3), (2, 0, 1), None, torch.float32), ((33, 65, 1), (0, 1, 2), 72, torch.float32),
             ((100, 200, 1), (1, 0, 2), 104, torch.bfloat16), ((36, 44, 1), (0, 1, 2), 48, torch.float32),
             ((36, 44, 1), (1, 0, 2), 40, torch.float32)]   # partial 32 x 32 tiles on the 4-element path
    jobs, want = [], []
    for (d0, d1, d2), pm, pitch, dt in specs:
        src = torch.randn(d0, d1, d2, device=gpu, generator=g)
        ref = src.permute(*pm).contiguous()
        od = ref.shape
        if pitch is None:
            dst = torch.full((ref.numel(),), float("nan"), device=gpu, dtype=dt)
            want.append((dst, ref.to(dt).reshape(-1), None))
        else:   # padded [od0][pitch] destination, the padding left alone (zeros here)
            dst = torch.zeros(od[0] * pitch, device=gpu, dtype=dt)
            full = torch.zeros(od[0], pitch, device=gpu, dtype=dt)
            full[:, :od[1] * od[2]] = ref.reshape(od[0], -1).to(dt)
            want.append((dst, full.reshape(-1), None))
        jobs.append((src.reshape(-1), dst, d0, d1, d2, pm, pitch))
    ops.PermuteBatch().run(jobs)
    torch.cuda.synchronize()
    for dst, ref, _ in want:
        assert torch.equal(dst, ref)


@pytest.mark.parametrize("CIN,COUT", [(64, 128), (128, 128), (128, 256)])
@pytest.mark.parametrize("act", [0, 1, 2])
@pytest.mark.parametrize("N,H,W", [(2, 147, 147), (3, 9, 150), (5, 1, 152), (2, 6, 3), (1, 300, 37), (600, 3, 20),
                                   (2, 74, 74), (3, 5, 78)])
def test_sep_fwd_vs_dw_and_gemm(ops, gpu, N, H, W, CIN, COUT, act):
    """Fused depthwise + pointwise forward of block1's units and block2's first (csrc/sepfwd.hip) against
    the two kernels it replaces: D bitwise xcp_dw_fwd's, Y bitwise the NT GEMM's (same MFMA operands and K
    order; the 128x128 kernel for 128 outputs, the persistent 256x256 one for 256), the BN partial sums to
    fp32 summation order against the NT epilogue's; frames as wide as each form takes, one row, three
    columns (W <= 8 powers of two take dwframe.hip, fp32 windows), fewer tiles than workgroups and more
    (600 frames: a workgroup walks several frames, its look-ahead loads crossing tile boundaries)."""
    if COUT == 256 and W > 78:
        pytest.skip("the 256-output form takes frames up to 78 wide")
    g = torch.Generator(device=gpu).manual_seed(N * 1000 + H + W + CIN + COUT + act)
    M = N * H * W
    X = torch.randn(M, CIN, device=gpu, generator=g).bfloat16()
    sc = torch.rand(CIN, device=gpu, generator=g) + 0.5
    sh = torch.randn(CIN, device=gpu, generator=g) * 0.5
    dwt = torch.randn(9, CIN, device=gpu, generator=g) * 0.3
    pw = (torch.randn(COUT, CIN, device=gpu, generator=g) / CIN ** 0.5).bfloat16()
    D_ref = torch.empty(M, CIN, device=gpu, dtype=torch.bfloat16)
    ops.dw_fwd(act, X, D_ref, dwt, sc, sh, N, H, W, CIN)
    Y_ref = torch.empty(M, COUT, device=gpu, dtype=torch.bfloat16)
    R_ref = ops.nt_stat_rows(M)
    part_ref = torch.zeros(R_ref * 2 * COUT, device=gpu)
    ops.gemm_nt(D_ref, pw, Y_ref, M, COUT, CIN, stats=part_ref)
    R = ops.sep_fwd_parts(torch.bfloat16, N, H, W, CIN, COUT)
    assert 0 < R <= min(N * H, torch.cuda.get_device_properties(gpu).multi_processor_count)
    D = torch.full((M, CIN), float("nan"), device=gpu, dtype=torch.bfloat16)
    Y = torch.full((M, COUT), float("nan"), device=gpu, dtype=torch.bfloat16)
    part = torch.full((R * 2 * COUT,), float("nan"), device=gpu)
    ops.sep_fwd(act, X, sc, sh, dwt, pw, D, Y, part, N, H, W, CIN, COUT)
    torch.cuda.synchronize()
    assert torch.equal(D, D_ref)
    assert torch.equal(Y, Y_ref)
    sums = part.view(R, 2, COUT).double().sum(0)
    sums_ref = part_ref.view(R_ref, 2, COUT).double().sum(0)
    yd = Y_ref.double()
    exact = torch.stack([yd.sum(0), (yd * yd).sum(0)])
    scale = torch.stack([yd.abs().sum(0), (yd * yd).sum(0)]) + 1e-30
    assert ((sums - exact).abs() / scale).max().item() < 2e-6
    assert ((sums_ref - exact).abs() / scale).max().item() < 2e-6


def test_sep_fwd_rejects_unsupported(ops, gpu):
    assert ops.sep_fwd_parts(torch.bfloat16, 2, 8, 153, 64, 128) == 0   # wider than 152
    assert ops.sep_fwd_parts(torch.bfloat16, 2, 8, 8, 256, 128) == 0
    assert ops.sep_fwd_parts(torch.bfloat16, 2, 8, 8, 64, 256) == 0
    assert ops.sep_fwd_parts(torch.bfloat16, 2, 8, 79, 128, 256) == 0   # the 256-output form: one half row
    assert ops.sep_fwd_parts(torch.bfloat16, 2, 8, 8, 256, 256) == 0
    assert ops.sep_fwd_parts(torch.float32, 2, 8, 8, 64, 128) == 0


@pytest.mark.parametrize("M,N,K", [(92416, 728, 728), (3000, 296, 520), (32 * 7 + 5, 256, 264), (20000, 1024, 256)])
def test_gemm_tn_loops_bitwise(ops, gpu, monkeypatch, M, N, K):
    """The weight-gradient kernel with one 32-MFMA phase per step and the fill four steps ahead
    (gemm_tn256q_kernel, the default) against gemm_tn256_kernel (XCP_TN_LOOP=1): the same MFMA order per
    accumulator, so the fp32 partial slabs are bitwise equal (ragged M / N / K, splits shorter than
    the ring)."""
    g = torch.Generator(device=gpu).manual_seed(M + N + K)
    G = torch.randn(M, N, device=gpu, generator=g).bfloat16()
    X = torch.randn(M, K, device=gpu, generator=g).bfloat16()
    rps = ops._lib.call("xcp_gemm_tn_rows_per_split", 1, 0, M, N, K, 2)
    S = (M + rps - 1) // rps
    outs = []
    for form in ("1", "2"):
        monkeypatch.setenv("XCP_TN_LOOP", form)
        P = torch.full((S * N * K,), float("nan"), device=gpu)
        ops.gemm_tn(G, X, P, M, N, K, S, rps, tile=2)
        torch.cuda.synchronize()
        outs.append(P)
    assert not torch.isnan(outs[1]).any()
    assert torch.equal(outs[0], outs[1])
    ref = (G.float().t() @ X.float())
    got = outs[1].view(S, N, K).sum(0)
    torch.testing.assert_close(got, ref, rtol=2e-3, atol=2e-3 * ref.abs().max().item())


@pytest.mark.parametrize("form", ["XCP_NT_HALF", "XCP_NT_PF2", "XCP_NT_4W", "XCP_NT_8W", "XCP_NT_KHALF"])
@pytest.mark.parametrize("M,N,K,stats", [(92416, 736, 736, True), (92416, 736, 736, False), (256 * 100 + 7, 768, 200, True),
                                         (256 * 100 + 7, 768, 392, False), (256 * 300 + 5, 512, 128, False),
                                         (256 * 100 + 7, 736, 728, True)])
def test_gemm_nt_half_tiles_bitwise(ops, gpu, monkeypatch, M, N, K, stats, form):
    """XCP_NT_HALF=1: the persistent kernel walks the last round's tiles as two half tiles each (only one
    B half's quadrants and columns per half) before the whole tiles; XCP_NT_PF2=1: it issues the next tile's
    first two K-tiles ahead of each epilogue (K = 128: two K-tiles, every wait of the second one's form);
    XCP_NT_4W=1: the one-wave-per-SIMD kernel (gemm_nt4w_kernel; K = 200 / 392 / 736: an odd number of
    32-deep steps, padded by a step of zero fragments); XCP_NT_KHALF (0 in the reference run, 1 = the default):
    a last K-tile with K % 64 in (0, 32] multiplies its first 32-deep half only (K = 200 / 392 / 728 / 736) --
    with the static walk (statistics) and with the tile queue (none): output and statistics bits identical
    to the reference run for every row: the one-shot kernel for the half tiles (every row on the persistent
    kernel), the default persistent kernel (same sparse last round on the 128x128 kernel) for the others."""
    g = torch.Generator(device=gpu).manual_seed(M + N + K)
    A = torch.randn(M, K, device=gpu, generator=g).bfloat16()
    B = (torch.randn(N, K, device=gpu, generator=g) / K ** 0.5).bfloat16()
    R = ops.nt_stat_rows(M)
    outs = []
    for i, t in enumerate((2 if form == "XCP_NT_HALF" else 0, 0, 0)):   # (twice: the tile queue's counter must be reset)
        monkeypatch.setenv(form, "1" if i else "0")
        C = torch.full((M, N), float("nan"), device=gpu, dtype=torch.bfloat16)
        part = torch.full((R, 2, N), float("nan"), device=gpu) if stats else None
        ops.gemm_nt(A, B, C, M, N, K, stats=part, tile=t)
        torch.cuda.synchronize()
        outs.append((C, part))
    torch.cuda.synchronize()
    for C, part in outs[1:]:
        assert torch.equal(outs[0][0], C)
        if stats:
            assert torch.equal(outs[0][1], part)
