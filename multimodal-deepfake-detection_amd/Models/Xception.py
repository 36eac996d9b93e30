"""Xception (Chollet 2017) backbone -- module surface of the reference, MI355X engine underneath.

Mirrors /root/reference/Xception.py: same classes (``SeparableConv2d``
:37-47, ``Block`` :50-99, ``Xception`` :102-201, ``xception()`` :205-213), same
submodule names and registration order, same init (:154-160, identical RNG
consumption), hence identical ``state_dict`` keys/shapes and bit-identical
seeded init.  The convolutions, BatchNorms and max-pools are the ``xcp.modules``
subclasses of the torch.nn classes, whose forward runs the ``torch.ops.xcp.*`` custom
ops, so every sub-module (``model.block4``, ``SeparableConv2d``, ``Block``) runs on its
own as in the reference.  ``Xception.forward`` runs the whole backbone as ONE fused
pass of the gfx950 kernels (``xcp.engine``, one autograd node); when forward hooks or
pre-hooks are registered on any sub-module it composes the sub-modules instead (the
reference's Xception.py:167-201 order), so the hooks fire.  There is no CPU path: a
non-GPU input raises.

Offline: ``xception(pretrained=True)`` never fetches (the reference downloads
from data.lip6.fr, Xception.py:33,212).  It loads a local copy named by
``pretrained=<path>`` or ``$XCP_XCEPTION_WEIGHTS`` (or the torch hub cache) with
``torch.load(weights_only=True)`` and raises if none is present.
"""
import math
import os

import torch
import torch.nn as nn
import torch.nn.functional as F

from xcp import modules as xm

__all__ = ["xception"]

model_urls = {"xception": "http://data.lip6.fr/cadene/pretrainedmodels/xception-43020ad28.pth"}


class SeparableConv2d(nn.Module):
    """depthwise kxk (groups=C) followed by pointwise 1x1 (Xception.py:37-47)."""

    def __init__(self, in_channels, out_channels, kernel_size=1, stride=1, padding=0, dilation=1, bias=False):
        super(SeparableConv2d, self).__init__()
        self.conv1 = xm.DepthwiseConv2d(in_channels, in_channels, kernel_size, stride, padding, dilation,
                                        groups=in_channels, bias=bias)
        self.pointwise = xm.PointwiseConv2d(in_channels, out_channels, 1, 1, 0, 1, 1, bias=bias)

    def forward(self, x):   # Xception.py:44-47
        x = self.conv1(x)
        x = self.pointwise(x)
        return x


class Block(nn.Module):
    """Xception block (Xception.py:50-99): [ReLU -> SepConv -> BN] x reps, optional MaxPool,
    plus identity or 1x1-conv+BN skip."""

    def __init__(self, in_filters, out_filters, reps, strides=1, start_with_relu=True, grow_first=True):
        super(Block, self).__init__()
        if out_filters != in_filters or strides != 1:
            self.skip = xm.PointwiseConv2d(in_filters, out_filters, 1, stride=strides, bias=False)
            self.skipbn = xm.BatchNorm2d(out_filters)
        else:
            self.skip = None
        self.relu = nn.ReLU(inplace=True)
        rep = []
        filters = in_filters
        if grow_first:
            rep.append(self.relu)
            rep.append(SeparableConv2d(in_filters, out_filters, 3, stride=1, padding=1, bias=False))
            rep.append(xm.BatchNorm2d(out_filters))
            filters = out_filters
        for _ in range(reps - 1):
            rep.append(self.relu)
            rep.append(SeparableConv2d(filters, filters, 3, stride=1, padding=1, bias=False))
            rep.append(xm.BatchNorm2d(filters))
        if not grow_first:
            rep.append(self.relu)
            rep.append(SeparableConv2d(in_filters, out_filters, 3, stride=1, padding=1, bias=False))
            rep.append(xm.BatchNorm2d(out_filters))
        if not start_with_relu:
            rep = rep[1:]
        else:
            rep[0] = nn.ReLU(inplace=False)
        if strides != 1:
            rep.append(xm.MaxPool2d(3, strides, 1))
        self.rep = nn.Sequential(*rep)

    def forward(self, inp):   # Xception.py:89-99
        x = self.rep(inp)
        if self.skip is not None:
            skip = self.skip(inp)
            skip = self.skipbn(skip)
        else:
            skip = inp
        x += skip
        return x


class Xception(nn.Module):
    """Xception-41 feature extractor + fc (Xception.py:102-201)."""

    def __init__(self, num_classes=1000):
        super(Xception, self).__init__()
        self.num_classes = num_classes
        self.conv1 = xm.StemConv2d(3, 32, 3, 2, 0, bias=False)
        self.bn1 = xm.BatchNorm2d(32)
        self.relu = nn.ReLU(inplace=True)
        self.conv2 = xm.StemConv2d(32, 64, 3, bias=False)
        self.bn2 = xm.BatchNorm2d(64)
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
        self.bn3 = xm.BatchNorm2d(1536)
        self.conv4 = SeparableConv2d(1536, 2048, 3, 1, 1)
        self.bn4 = xm.BatchNorm2d(2048)
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
        self._xcp_grad_sink = None   # xcp.ddp.GradBuckets(module=...) registers itself here
        self._xcp_buffer_wait = None   # xcp.ddp.broadcast_buffers' completion event (async form)
        self.register_state_dict_pre_hook(_wait_buffers_hook)   # a checkpoint reads broadcast values

    def _xcp_wait_buffers(self):
        """Make the current stream wait for a pending buffer broadcast (xcp.ddp.broadcast_buffers),
        once: called where the forward first touches a BatchNorm running statistic."""
        ev = getattr(self, "_xcp_buffer_wait", None)
        if ev is not None:
            self._xcp_buffer_wait = None
            torch.cuda.current_stream(self.conv1.weight.device).wait_event(ev)

    def _engine(self):
        from xcp import compute_dtype
        from xcp.engine import XceptionEngine
        dt = compute_dtype()
        eng = self._xcp_engines.get(dt)
        if eng is None or eng.model is not self:
            # (a shallow copy of this module -- e.g. an nn.DataParallel replica made before
            # _replicate_for_data_parallel below existed -- never drives another module's engine)
            if eng is not None:
                self._xcp_engines = {}
            eng = self._xcp_engines[dt] = XceptionEngine(self, dt)
        return eng

    def _replicate_for_data_parallel(self):
        """nn.DataParallel replica (train_audio.py:16-18): its own engine cache (an engine holds
        the module it packs weights from) and no gradient sink -- a replica's gradients reach
        the original parameters through DataParallel's autograd broadcast."""
        self._xcp_wait_buffers()   # replicas copy the buffers as broadcast
        r = super()._replicate_for_data_parallel()
        r._xcp_engines = {}
        r._xcp_grad_sink = None
        r._xcp_buffer_wait = None
        return r

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

    def _hooked(self):
        """True when a forward (pre-)hook is registered on a sub-module or globally: the fused
        engine would skip those modules' forward calls, so the module path runs instead."""
        from torch.nn.modules import module as _m
        if _m._global_forward_hooks or _m._global_forward_pre_hooks:
            return True
        return any(m._forward_hooks or m._forward_pre_hooks for m in self.modules() if m is not self)

    def forward_modules(self, x):
        """Xception.forward as the reference composes it (Xception.py:167-201), each sub-module on
        the xcp custom ops.  Returns fp32 features through ``fc``."""
        x = self.conv1(x)
        self._xcp_wait_buffers()   # (xcp.ddp.broadcast_buffers) first running-statistic access
        x = self.bn1(x)
        x = self.relu(x)
        x = self.conv2(x)
        x = self.bn2(x)
        x = self.relu(x)
        for i in range(1, 13):
            x = getattr(self, f"block{i}")(x)
        x = self.conv3(x)
        x = self.bn3(x)
        x = self.relu(x)
        x = self.conv4(x)
        x = self.bn4(x)
        x = self.relu(x)
        x = F.adaptive_avg_pool2d(x, (1, 1))
        x = x.reshape(x.size(0), -1).float()
        return self.fc(x)

    def forward(self, x):
        if self._hooked():
            return self.forward_modules(x)
        return self.fc(self.features(x))

    def __getstate__(self):   # copies (torch.save, deepcopy for AveragedModel) share no engine / sink
        self._xcp_wait_buffers()
        d = self.__dict__.copy()
        d["_xcp_engines"] = {}
        d["_xcp_grad_sink"] = None
        d["_xcp_buffer_wait"] = None
        return d


def _wait_buffers_hook(module, prefix, keep_vars):
    module._xcp_wait_buffers()


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
