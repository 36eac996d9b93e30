"""Xception (Chollet 2017) backbone -- module surface of the reference, MI355X engine underneath.

Mirrors /root/reference/Xception.py: same classes (``SeparableConv2d``
:37-47, ``Block`` :50-99, ``Xception`` :102-201, ``xception()`` :205-213), same
submodule names and registration order, same init (:154-160, identical RNG
consumption), hence identical ``state_dict`` keys/shapes and bit-identical
seeded init.  ``Xception.forward`` runs the whole backbone on the hand-written
gfx950 kernels through ``xcp.engine`` (one autograd node); there is no CPU
path -- a non-GPU input raises.

Offline: ``xception(pretrained=True)`` never fetches (the reference downloads
from data.lip6.fr, Xception.py:33,212).  It loads a local copy named by
``pretrained=<path>`` or ``$XCP_XCEPTION_WEIGHTS`` (or the torch hub cache) with
``torch.load(weights_only=True)`` and raises if none is present.
"""
import math
import os

import torch
import torch.nn as nn

__all__ = ["xception"]

model_urls = {"xception": "http://data.lip6.fr/cadene/pretrainedmodels/xception-43020ad28.pth"}


class SeparableConv2d(nn.Module):
    """depthwise kxk (groups=C) followed by pointwise 1x1 (Xception.py:37-47)."""

    def __init__(self, in_channels, out_channels, kernel_size=1, stride=1, padding=0, dilation=1, bias=False):
        super(SeparableConv2d, self).__init__()
        self.conv1 = nn.Conv2d(in_channels, in_channels, kernel_size, stride, padding, dilation, groups=in_channels,
                               bias=bias)
        self.pointwise = nn.Conv2d(in_channels, out_channels, 1, 1, 0, 1, 1, bias=bias)

    def forward(self, x):
        raise RuntimeError("SeparableConv2d runs inside the fused xcp Xception engine; call the Xception module "
                           "(per-module execution is not provided on MI355X)")


class Block(nn.Module):
    """Xception block (Xception.py:50-99): [ReLU -> SepConv -> BN] x reps, optional MaxPool,
    plus identity or 1x1-conv+BN skip."""

    def __init__(self, in_filters, out_filters, reps, strides=1, start_with_relu=True, grow_first=True):
        super(Block, self).__init__()
        if out_filters != in_filters or strides != 1:
            self.skip = nn.Conv2d(in_filters, out_filters, 1, stride=strides, bias=False)
            self.skipbn = nn.BatchNorm2d(out_filters)
        else:
            self.skip = None
        self.relu = nn.ReLU(inplace=True)
        rep = []
        filters = in_filters
        if grow_first:
            rep.append(self.relu)
            rep.append(SeparableConv2d(in_filters, out_filters, 3, stride=1, padding=1, bias=False))
            rep.append(nn.BatchNorm2d(out_filters))
            filters = out_filters
        for _ in range(reps - 1):
            rep.append(self.relu)
            rep.append(SeparableConv2d(filters, filters, 3, stride=1, padding=1, bias=False))
            rep.append(nn.BatchNorm2d(filters))
        if not grow_first:
            rep.append(self.relu)
            rep.append(SeparableConv2d(in_filters, out_filters, 3, stride=1, padding=1, bias=False))
            rep.append(nn.BatchNorm2d(out_filters))
        if not start_with_relu:
            rep = rep[1:]
        else:
            rep[0] = nn.ReLU(inplace=False)
        if strides != 1:
            rep.append(nn.MaxPool2d(3, strides, 1))
        self.rep = nn.Sequential(*rep)

    def forward(self, inp):
        raise RuntimeError("Block runs inside the fused xcp Xception engine; call the Xception module")


class Xception(nn.Module):
    """Xception-41 feature extractor + fc (Xception.py:102-201)."""

    def __init__(self, num_classes=1000):
        super(Xception, self).__init__()
        self.num_classes = num_classes
        self.conv1 = nn.Conv2d(3, 32, 3, 2, 0, bias=False)
        self.bn1 = nn.BatchNorm2d(32)
        self.relu = nn.ReLU(inplace=True)
        self.conv2 = nn.Conv2d(32, 64, 3, bias=False)
        self.bn2 = nn.BatchNorm2d(64)
        self.block1 = Block(64, 128, 2, 2, start_with_relu=False, grow_first=True)
        self.block2 = Block(128, 256, 2, 2, start_with_relu=True, grow_first=True)
        self.block3 = Block(256, 728, 2, 2, start_with_relu=True, grow_first=True)
        self.block4 = Block(728, 728, 3, 1, start_with_relu=True, grow_first=True)
        self.block5 = Block(728, 728, 3, 1, start_with_relu=True, grow_first=True)
        self.block6 = Block(728, 728, 3, 1, start_with_relu=True, grow_first=True)
        self.block7 = Block(728, 728, 3, 1, start_with_relu=True, grow_first=True)
        self.block8 = Block(728, 728, 3, 1, start_with_relu=True, grow_first=True)
        self.block9 = Block(728, 728, 3, 1, start_with_relu=True, grow_first=True)
        self.block10 = Block(728, 728, 3, 1, start_with_relu=True, grow_first=True)
        self.block11 = Block(728, 728, 3, 1, start_with_relu=True, grow_first=True)
        self.block12 = Block(728, 1024, 2, 2, start_with_relu=True, grow_first=False)
        self.conv3 = SeparableConv2d(1024, 1536, 3, 1, 1)
        self.bn3 = nn.BatchNorm2d(1536)
        self.conv4 = SeparableConv2d(1536, 2048, 3, 1, 1)
        self.bn4 = nn.BatchNorm2d(2048)
        self.fc = nn.Linear(2048, num_classes)
        # ------- init weights (Xception.py:154-160) --------
        for m in self.modules():
            if isinstance(m, nn.Conv2d):
                n = m.kernel_size[0] * m.kernel_size[1] * m.out_channels
                m.weight.data.normal_(0, math.sqrt(2. / n))
            elif isinstance(m, nn.BatchNorm2d):
                m.weight.data.fill_(1)
                m.bias.data.zero_()
        self._xcp_engines = {}

    def _engine(self):
        from xcp import compute_dtype
        from xcp.engine import XceptionEngine
        dt = compute_dtype()
        eng = self._xcp_engines.get(dt)
        if eng is None:
            eng = self._xcp_engines[dt] = XceptionEngine(self, dt)
        return eng

    def features(self, x):
        """Backbone up to the global average pool: [N,3,H,W] fp32 -> [N,2048] fp32."""
        from xcp import ops
        from xcp.engine import XceptionFunction
        ops.check_gpu(x)
        eng = self._engine()
        params = [p for _, p in eng.named_params()]
        if torch.is_grad_enabled() and any(p.requires_grad for p in params):
            return XceptionFunction.apply(eng, self.training, x, *params)
        feats, _ = eng.forward(x, self.training)
        return feats

    def forward(self, x):
        return self.fc(self.features(x))

    def __getstate__(self):
        d = self.__dict__.copy()
        d["_xcp_engines"] = {}
        return d


def _local_weights(pretrained):
    if isinstance(pretrained, (str, os.PathLike)):
        return str(pretrained)
    cands = [os.environ.get("XCP_XCEPTION_WEIGHTS", "")]
    hub = os.path.join(torch.hub.get_dir(), "checkpoints", os.path.basename(model_urls["xception"]))
    cands.append(hub)
    for c in cands:
        if c and os.path.exists(c):
            return c
    raise RuntimeError("xception(pretrained=True): no local copy of xception-43020ad28.pth (set "
                       "XCP_XCEPTION_WEIGHTS or pass a path); this build never downloads weights")


def xception(pretrained=False, **kwargs):
    """Construct Xception (Xception.py:205-213)."""
    model = Xception(**kwargs)
    if pretrained:
        sd = torch.load(_local_weights(pretrained), map_location="cpu", weights_only=True)
        model.load_state_dict(sd)
    return model
