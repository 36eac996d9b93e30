"""The module-level boundary: Xception's sub-modules run on their own through the
torch.library ops in namespace ``xcp`` (xcp/torch_ops.py, xcp/modules.py), against the
reference's golden vectors (tests/golden, captured from the reference modules themselves).

Tolerances as tests/test_gpu_model.py: fp32 rel 1e-4 (values) / 1e-3 (gradient norms);
bf16 cosine >= 0.999 on outputs and >= 0.99 on input gradients.
"""
import numpy as np
import pytest
import torch
import torch.nn as nn

pytestmark = pytest.mark.gpu


def seeded_normal(shape, seed):
    return torch.randn(shape, generator=torch.Generator().manual_seed(seed), dtype=torch.float32)


def cos(a, b):
    a, b = np.asarray(a, np.float64).ravel(), np.asarray(b, np.float64).ravel()
    return float(a @ b / (np.linalg.norm(a) * np.linalg.norm(b)))


def check_fp(g, prefix, t, f32, rtol=1e-4, min_cos=0.999, flips=0.0):
    """fingerprint check; ``flips``: fraction of sampled elements allowed outside the tolerance
    (input gradients of pooled blocks: a max-pool argmax tie broken differently by a last-bit
    difference routes a whole gradient to a neighbouring pixel)."""
    a = t.detach().double().reshape(-1).cpu().numpy()
    assert tuple(g[f"{prefix}/shape"]) == tuple(t.shape)
    if f32:
        got, want = a[g[f"{prefix}/idx"]], g[f"{prefix}/val"]
        bad = np.abs(got - want) > 1e-5 + rtol * np.abs(want)
        assert bad.mean() <= flips, (prefix, bad.mean())
        np.testing.assert_allclose((a * a).sum(), g[f"{prefix}/sumsq"], rtol=rtol if not flips else 2e-2)
    else:
        assert cos(a[g[f"{prefix}/idx"]], g[f"{prefix}/val"]) > min_cos


def init_like_xception(mod):
    for mm in mod.modules():   # Xception.py:154-160
        if isinstance(mm, nn.Conv2d):
            n = mm.kernel_size[0] * mm.kernel_size[1] * mm.out_channels
            mm.weight.data.normal_(0, (2.0 / n) ** 0.5)


@pytest.mark.parametrize("prec", ["fp32", "bf16"])
def test_separable_conv_module(gpu, golden, prec):
    """SeparableConv2d.forward (Xception.py:44-47) = xcp::dwconv3x3 + xcp::pointwise, every
    distinct backbone shape, forward and backward, against sepconv.npz."""
    from Models.Xception import SeparableConv2d
    g = golden("sepconv.npz")
    f32 = prec == "fp32"
    dt = torch.float32 if f32 else torch.bfloat16
    for key in sorted({k.split("/")[0] for k in g if k.startswith("s")}):
        cin, cout, hw, sw, sx, sr = [int(v) for v in g[f"{key}/cfg"]]
        torch.manual_seed(sw)
        sc = SeparableConv2d(cin, cout, 3, 1, 1).to(gpu)
        x = seeded_normal((2, cin, hw, hw), sx).to(gpu).to(dt).requires_grad_(True)
        y = sc(x)
        assert y.dtype == dt and y.shape == (2, cout, hw, hw)
        (y.float() * seeded_normal(y.shape, sr).to(gpu)).sum().backward()
        torch.cuda.synchronize()
        check_fp(g, f"{key}/y", y.float(), f32)
        check_fp(g, f"{key}/dx", x.grad.float(), f32, min_cos=0.99)
        dwg = sc.conv1.weight.grad.cpu().numpy()
        if f32:
            np.testing.assert_allclose(dwg, g[f"{key}/dw_grad"], rtol=1e-3, atol=1e-4)
            np.testing.assert_allclose(sc.pointwise.weight.grad.double().norm().item(), g[f"{key}/pw_gradnorm"],
                                       rtol=1e-4)
        else:
            assert cos(dwg, g[f"{key}/dw_grad"]) > 0.99
            np.testing.assert_allclose(sc.pointwise.weight.grad.double().norm().item(), g[f"{key}/pw_gradnorm"],
                                       rtol=5e-2)


@pytest.mark.parametrize("prec", ["fp32", "bf16"])
def test_block_module(gpu, golden, prec):
    """Block.forward (Xception.py:89-99: rep with ReLU / SeparableConv2d / BatchNorm2d (train) /
    MaxPool2d, skip conv + BN, x += skip) for block1 (stride 2, no leading ReLU), block4
    (identity skip) and block12 (grow_first=False), against blocks.npz, including the BN
    running statistics after the call."""
    from Models.Xception import Block
    g = golden("blocks.npz")
    f32 = prec == "fp32"
    dt = torch.float32 if f32 else torch.bfloat16
    for i, name in enumerate(["block1", "block4", "block12"]):
        cin, cout, reps, s, swr, gf, hw = [int(v) for v in g[f"{name}/cfg"]]
        torch.manual_seed(10 + i)
        blk = Block(cin, cout, reps, s, start_with_relu=bool(swr), grow_first=bool(gf))
        init_like_xception(blk)
        blk = blk.to(gpu).train()
        x = seeded_normal((2, cin, hw, hw), 100 + i).to(gpu).to(dt).requires_grad_(True)
        y = blk(x)
        (y.float() * seeded_normal(y.shape, 200 + i).to(gpu)).sum().backward()
        torch.cuda.synchronize()
        check_fp(g, f"{name}/out", y.float(), f32)
        check_fp(g, f"{name}/dx", x.grad.float(), f32, rtol=1e-3, min_cos=0.99, flips=0.02 if s != 1 else 0.0)
        errs = {}
        for n, p in blk.named_parameters():
            key = f"{name}/gradnorm/{n}"
            if key in g:
                e = abs(p.grad.double().norm().item() - g[key]) / g[key]
                errs[n] = e
                if f32:
                    assert e < (5e-3 if p.dim() == 1 else 1e-3), (name, n, e)
        if not f32:   # SURVEY 8c's 5e-2 with the measured exceptions (tests/bf16_contract.py)
            import bf16_contract
            bf16_contract.check(f"blocks_{name}", errs)
        for n, t in blk.state_dict().items():
            if "running" in n:
                np.testing.assert_allclose(t.double().sum().item(), g[f"{name}/buf/{n}/sum"],
                                           rtol=1e-4 if f32 else 3e-2, atol=1e-5 if f32 else 3e-2, err_msg=n)


def test_forward_hooks_use_module_path(gpu):
    """A forward hook on a sub-module makes Xception.forward compose the sub-modules (the
    reference's order), so the hook fires; the result equals the fused engine's (fp32), and so
    do the parameter gradients."""
    import xcp
    from Models.Xception import xception
    torch.manual_seed(0)
    m = xception(num_classes=1000)
    m.fc = nn.Identity()
    m = m.to(gpu).train()
    x = torch.rand((2, 3, 96, 96), generator=torch.Generator().manual_seed(3)).to(gpu)
    with xcp.precision("fp32"):
        f_engine = m(x)
        f_engine.sum().backward()
        g_engine = {n: p.grad.clone() for n, p in m.named_parameters()}
        m.zero_grad()
        seen = []
        h = m.block4.rep[1].register_forward_hook(lambda mod, i, o: seen.append(tuple(o.shape)))
        f_mod = m(x)
        f_mod.sum().backward()
        h.remove()
    torch.cuda.synchronize()
    assert seen == [(2, 728, 6, 6)]
    torch.testing.assert_close(f_mod, f_engine, rtol=1e-4, atol=1e-5)
    # two fp32 evaluations of the graph (fused BN-on-load vs materialised per-module tensors) differ in
    # summation order; through 40 BatchNorms that spreads to ~3e-3 on a weight gradient, as the
    # reference's own fp32 result differs from fp64 (test_gpu_model fp32 contract: 1e-3 / 5e-3 per norm)
    for n, p in m.named_parameters():
        a, b = p.grad.double(), g_engine[n].double()
        assert ((a - b).norm() / b.norm().clamp_min(1e-30)).item() < (1e-2 if p.dim() == 1 else 5e-3), n


def test_opcheck_xcp_ops(gpu):
    """torch.library.opcheck: schema, fake (meta) kernels, autograd registration of the ops."""
    from xcp import torch_ops  # noqa: F401
    g = torch.Generator(device=gpu).manual_seed(0)

    def r(*shape, dt=torch.float32, grad=False):
        return torch.randn(shape, device=gpu, generator=g, dtype=torch.float32).to(dt).requires_grad_(grad)

    x = r(2, 64, 9, 10, grad=True)
    cases = [
        (torch.ops.xcp.dwconv3x3, (x, r(64, 1, 3, 3, grad=True))),
        (torch.ops.xcp.pointwise, (x, r(128, 64, 1, 1, grad=True), 1)),
        (torch.ops.xcp.pointwise, (x, r(128, 64, 1, 1, grad=True), 2)),
        (torch.ops.xcp.batch_norm, (x, r(64, grad=True), r(64, grad=True), torch.zeros(64, device=gpu),
                                    torch.ones(64, device=gpu), True, 0.1, 1e-5)),
        (torch.ops.xcp.max_pool3x3s2, (x,)),
        (torch.ops.xcp.stem_conv2, (r(2, 32, 9, 9, grad=True), r(64, 32, 3, 3, grad=True))),
        (torch.ops.xcp.lstm, (r(2, 5, 64, grad=True), r(512, 64, grad=True), r(512, 128, grad=True),
                              r(512, grad=True), r(512, grad=True), 0)),
    ]
    for op, args in cases:
        torch.library.opcheck(op, args, test_utils=("test_schema", "test_faketensor", "test_autograd_registration"))


@pytest.mark.parametrize("training", [True, False])
def test_batchnorm_module_backward(gpu, training):
    """xcp.modules.BatchNorm2d (Xception.py:56 and every rep BN) forward + backward against
    nn.BatchNorm2d in fp32, in training (batch statistics) and eval mode (running statistics: the
    input gradient is the affine map, dgamma / dbeta from the BN reduce and the colreduce slab sum)."""
    from xcp.modules import BatchNorm2d
    torch.manual_seed(3)
    C = 40
    ref = nn.BatchNorm2d(C).to(gpu)
    with torch.no_grad():
        ref.weight.uniform_(0.5, 1.5)
        ref.bias.normal_()
        ref.running_mean.normal_()
        ref.running_var.uniform_(0.5, 2.0)
    mine = BatchNorm2d(C).to(gpu)
    mine.load_state_dict(ref.state_dict())
    ref.train(training)
    mine.train(training)
    x = torch.randn(3, C, 9, 11, device=gpu)
    dy = torch.randn(3, C, 9, 11, device=gpu)
    xa, xb = x.clone().requires_grad_(True), x.clone().requires_grad_(True)
    ya, yb = ref(xa), mine(xb)
    ya.backward(dy)
    yb.backward(dy)
    torch.testing.assert_close(yb, ya, rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(xb.grad, xa.grad, rtol=1e-4, atol=1e-5)
    torch.testing.assert_close(mine.weight.grad, ref.weight.grad, rtol=1e-4, atol=1e-4)
    torch.testing.assert_close(mine.bias.grad, ref.bias.grad, rtol=1e-4, atol=1e-4)
