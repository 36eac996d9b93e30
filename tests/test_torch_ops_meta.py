"""CPU tests of the torch.library op layer (xcp/torch_ops.py): every op is registered in
namespace ``xcp`` with a fake kernel (shapes / dtypes / channels_last outputs on the meta
device, no GPU needed), and the module path refuses CPU tensors (no CPU fallback)."""
import pytest
import torch


def meta(*shape, dt=torch.float32):
    return torch.empty(shape, device="meta", dtype=dt)


def test_ops_registered():
    from xcp import torch_ops
    for name in torch_ops.OPS:
        assert hasattr(torch.ops.xcp, name), name


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
def test_fake_kernels(dt):
    from xcp import torch_ops  # noqa: F401
    x = meta(2, 64, 9, 10, dt=dt)
    y = torch.ops.xcp.dwconv3x3(x, meta(64, 1, 3, 3))
    assert y.shape == x.shape and y.dtype == dt and y.is_contiguous(memory_format=torch.channels_last)
    y = torch.ops.xcp.pointwise(x, meta(128, 64, 1, 1), 2)
    assert y.shape == (2, 128, 5, 5) and y.dtype == dt
    dx, dw = torch.ops.xcp.pointwise_backward(meta(2, 128, 5, 5, dt=dt), x, meta(128, 64, 1, 1), 2)
    assert dx.shape == x.shape and dw.shape == (128, 64, 1, 1) and dw.dtype == torch.float32
    y, mean, invstd, rm, rv = torch.ops.xcp.batch_norm(x, meta(64), meta(64), meta(64), meta(64), True, 0.1, 1e-5)
    assert y.shape == x.shape and mean.shape == (64,) and rm.shape == (64,)
    y, amax = torch.ops.xcp.max_pool3x3s2(x)
    assert y.shape == (2, 64, 5, 5) and amax.dtype == torch.uint8 and amax.numel() == 2 * 64 * 25
    y = torch.ops.xcp.stem_conv1(meta(2, 3, 299, 299), meta(32, 3, 3, 3), dt == torch.bfloat16)
    assert y.shape == (2, 32, 149, 149) and y.dtype == dt
    y = torch.ops.xcp.stem_conv2(meta(2, 32, 149, 149, dt=dt), meta(64, 32, 3, 3))
    assert y.shape == (2, 64, 147, 147)
    out = torch.ops.xcp.lstm(meta(4, 16, 2048), meta(512, 2048), meta(512, 128), meta(512), meta(512), 0)
    assert [tuple(t.shape) for t in out] == [(4, 16, 128), (1, 4, 128), (1, 4, 128), (4, 16, 128), (4, 16, 128),
                                             (4, 16, 512)]


def test_module_path_raises_on_cpu():
    from Models.Xception import Block, SeparableConv2d
    with pytest.raises(RuntimeError, match="MI355X"):
        Block(64, 64, 2, 1)(torch.zeros(1, 64, 8, 8))
    with pytest.raises(RuntimeError, match="MI355X"):
        SeparableConv2d(64, 128, 3, 1, 1)(torch.zeros(1, 64, 8, 8))
