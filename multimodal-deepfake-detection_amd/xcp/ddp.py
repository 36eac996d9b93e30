"""One-process-per-GPU data parallelism for the clip models (RCCL over xGMI).

Replaces the reference's single-process ``nn.DataParallel`` (train_audio.py:16-18,
which also bypasses DP for the backbone, :37).  Every rank owns a full replica
and a shard of the clip minibatch; the only exchange per step is the gradient
mean, done here as bucketed ``all_reduce`` calls (``"nccl"`` = RCCL on ROCm) on
one flat fp32 gradient buffer that the parameters' ``.grad`` tensors are views
of.  BatchNorm statistics stay per rank (the reference has no SyncBN); running
buffers are broadcast from rank 0 before each forward (DDP ``broadcast_buffers``
semantics).

Buckets are launched asynchronously as soon as every gradient in them has been
accumulated (post-accumulate-grad hooks): the head's (LSTM/FC) gradients arrive
first, so their all-reduce runs on RCCL's stream while the fused backbone
backward is still executing; the backbone buckets follow when the engine's
backward returns.  Parameters are laid out in the flat buffer in reverse
registration order so each bucket is contiguous.
"""
import torch
import torch.distributed as dist


class GradBuckets:
    def __init__(self, params, bucket_bytes=64 << 20, world=None):
        self.params = [p for p in params if p.requires_grad]
        self.world = world if world is not None else (dist.get_world_size() if dist.is_initialized() else 1)
        dev = self.params[0].device
        total = sum(p.numel() for p in self.params)
        self.flat = torch.zeros(total, device=dev, dtype=torch.float32)
        # reverse order: gradients of later layers are ready first
        off = 0
        self.views = {}
        for p in reversed(self.params):
            n = p.numel()
            v = self.flat[off:off + n].view_as(p)
            p.grad = v
            self.views[p] = (off, n)
            off += n
        # contiguous buckets over the flat buffer
        lim = max(1, bucket_bytes // 4)
        self.buckets = []
        start = 0
        cur = 0
        for p in reversed(self.params):
            o, n = self.views[p]
            if cur and cur + n > lim:
                self.buckets.append((start, start + cur))
                start, cur = o, 0
            cur += n
        if cur:
            self.buckets.append((start, start + cur))
        self._pending = []
        self._left = []
        self._bucket_of = {}
        for bi, (a, b) in enumerate(self.buckets):
            ps = [p for p in self.params if a <= self.views[p][0] < b]
            self._left.append(len(ps))
            for p in ps:
                self._bucket_of[p] = bi
        self._count = list(self._left)
        self.overlap = self.world > 1
        if self.overlap:
            for p in self.params:
                p.register_post_accumulate_grad_hook(self._on_grad)

    def _on_grad(self, p):
        bi = self._bucket_of[p]
        self._count[bi] -= 1
        if self._count[bi] == 0:
            a, b = self.buckets[bi]
            self._pending.append(dist.all_reduce(self.flat[a:b], op=dist.ReduceOp.SUM, async_op=True))

    def zero(self):
        self.flat.zero_()
        self._count = list(self._left)
        self._pending = []
        for p in self.params:  # re-attach if an optimizer set grads to None
            if p.grad is None or p.grad.data_ptr() != self.flat.data_ptr() + 4 * self.views[p][0]:
                o, n = self.views[p]
                p.grad = self.flat[o:o + n].view_as(p)

    def allreduce(self):
        """Finish the gradient mean across ranks (no-op at world size 1).  Buckets whose
        hooks did not fire (parameters without a gradient this step) are reduced here."""
        if self.world <= 1:
            return
        for bi, (a, b) in enumerate(self.buckets):
            if self._count[bi] != 0:
                self._count[bi] = 0
                self._pending.append(dist.all_reduce(self.flat[a:b], op=dist.ReduceOp.SUM, async_op=True))
        for w in self._pending:
            w.wait()
        self._pending = []
        self.flat.mul_(1.0 / self.world)


def broadcast_buffers(module, src=0):
    if not (dist.is_initialized() and dist.get_world_size() > 1):
        return
    bufs = [b for b in module.buffers() if b.is_floating_point()]
    if not bufs:
        return
    flat = torch.cat([b.reshape(-1) for b in bufs])
    dist.broadcast(flat, src)
    off = 0
    for b in bufs:
        n = b.numel()
        b.copy_(flat[off:off + n].view_as(b))
        off += n
