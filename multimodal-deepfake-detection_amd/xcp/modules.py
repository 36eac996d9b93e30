"""nn.Module subclasses whose forward runs the ``xcp`` custom ops (xcp.torch_ops).

Models/Xception.py builds the reference's module tree (Xception.py:37-160) from these in
place of ``nn.Conv2d`` / ``nn.BatchNorm2d`` / ``nn.MaxPool2d``.  They ARE those classes
(subclasses: same constructor, parameters, buffers, ``state_dict`` keys, init and RNG
consumption, and ``isinstance`` checks such as Xception.py:155-159 still hold); only
``forward`` changes, so a sub-module called on its own -- ``model.block4(x)``,
``sep.conv1(x)``, a forward hook on ``model.block4.rep[1]`` -- runs on the gfx950 kernels.
Configurations the Xception graph never uses raise ``NotImplementedError``.
"""
import torch
import torch.nn as nn

from . import torch_ops  # noqa: F401  (registers torch.ops.xcp.*)


def _check_cuda(x, what):
    if not x.is_cuda:
        raise RuntimeError(f"xcp {what} runs on the MI355X only (got a non-GPU tensor); there is no CPU fallback")


class DepthwiseConv2d(nn.Conv2d):
    """SeparableConv2d.conv1 (Xception.py:41): 3x3, stride 1, pad 1, groups = C, no bias."""

    def forward(self, x):
        _check_cuda(x, "depthwise conv")
        C = self.in_channels
        if (self.kernel_size, self.stride, self.padding, self.dilation, self.groups) != ((3, 3), (1, 1), (1, 1), (1, 1), C) \
                or self.out_channels != C or self.bias is not None or C % 8:
            raise NotImplementedError("xcp depthwise conv: 3x3 / stride 1 / pad 1 / groups=C / no bias, C % 8 == 0")
        return torch.ops.xcp.dwconv3x3(x, self.weight)


class PointwiseConv2d(nn.Conv2d):
    """SeparableConv2d.pointwise (Xception.py:42) and Block.skip (Xception.py:55): 1x1, no bias."""

    def forward(self, x):
        _check_cuda(x, "pointwise conv")
        if self.kernel_size != (1, 1) or self.padding != (0, 0) or self.groups != 1 or self.bias is not None \
                or self.stride[0] != self.stride[1] or self.in_channels % 8 or self.out_channels % 8:
            raise NotImplementedError("xcp pointwise conv: 1x1 / pad 0 / groups 1 / no bias, channels % 8 == 0")
        return torch.ops.xcp.pointwise(x, self.weight, self.stride[0])


class StemConv2d(nn.Conv2d):
    """Xception.conv1 (3 -> 32, 3x3 s2 p0, Xception.py:118) and conv2 (32 -> 64, 3x3 p0, :122)."""

    def forward(self, x):
        _check_cuda(x, "stem conv")
        from . import compute_dtype
        cfg = (self.in_channels, self.out_channels, self.kernel_size, self.stride, self.padding, self.bias is None)
        if cfg == (3, 32, (3, 3), (2, 2), (0, 0), True):
            return torch.ops.xcp.stem_conv1(x, self.weight, compute_dtype() == torch.bfloat16)
        if cfg == (32, 64, (3, 3), (1, 1), (0, 0), True):
            return torch.ops.xcp.stem_conv2(x, self.weight)
        raise NotImplementedError("xcp stem conv: Xception's conv1 (3->32 s2) / conv2 (32->64) only")


class BatchNorm2d(nn.BatchNorm2d):
    """nn.BatchNorm2d on xcp kernels (same training / eval / momentum semantics)."""

    def forward(self, x):
        _check_cuda(x, "batch norm")
        self._check_input_dim(x)
        if not self.affine or self.num_features % 8:
            raise NotImplementedError("xcp batch norm: affine, channels % 8 == 0")
        eaf = 0.0 if self.momentum is None else self.momentum
        if self.training and self.track_running_stats and self.num_batches_tracked is not None:
            self.num_batches_tracked.add_(1)
            eaf = 1.0 / float(self.num_batches_tracked) if self.momentum is None else self.momentum
        training = self.training or (self.running_mean is None and self.running_var is None)
        track = not self.training or self.track_running_stats
        rm = self.running_mean if track else None
        rv = self.running_var if track else None
        y, _, _, nrm, nrv = torch.ops.xcp.batch_norm(x, self.weight, self.bias, rm, rv, training, eaf, self.eps)
        if training and rm is not None:
            with torch.no_grad():
                rm.copy_(nrm)
                rv.copy_(nrv)
        return y


class MaxPool2d(nn.MaxPool2d):
    """Block's nn.MaxPool2d(3, 2, 1) (Xception.py:85-86)."""

    def forward(self, x):
        _check_cuda(x, "max pool")
        norm = lambda v: v if isinstance(v, tuple) else (v, v)   # noqa: E731
        if (norm(self.kernel_size), norm(self.stride), norm(self.padding), norm(self.dilation)) != \
                ((3, 3), (2, 2), (1, 1), (1, 1)) or self.ceil_mode or self.return_indices or x.shape[1] % 8:
            raise NotImplementedError("xcp max pool: MaxPool2d(3, 2, 1), channels % 8 == 0")
        return torch.ops.xcp.max_pool3x3s2(x)[0]
