"""The train_au_face.py training step (BASELINE config C5) on the xcp path.

``AUFaceTrainer`` holds what train_au_face.py:594-625 builds around the model and runs its
micro-step (:639-698) and evaluation step (:711-732):

* ``embed_head`` = LazyLinear(256) -> ReLU -> Dropout(0.2) -> Linear(256, 128) over the pooled
  [v_pool, au_pool] features; ``arcface`` = ArcFaceHead(128, 2, s=30, m=0.30) and ``cbfocal`` =
  CBFocalLoss(samples_per_cls, beta 0.9999, gamma 2) on the xcp heads kernels (xcp/heads.py);
* loss = CB-focal(ArcFace(embed)) + 0.2 * MSE(v_pool, au_pool) + 0.1 * temporal smoothness of
  both token streams (:666-674);
* gradient accumulation over ``accum_steps`` micro-batches (across ranks: one all-reduce of
  the flat gradient buffer on the micro-batch that steps, xcp/ddp.py), GradScaler (autocast: the xcp
  backbones run in bf16), unscale -> clip_grad_norm_(1.0) -> AdamW(lr 1e-4, wd 0.01) ->
  OneCycleLR(max_lr 1e-3, pct_start 0.3) -> AveragedModel updates of model and embed head
  (:678-693);
* evaluation with the averaged model and embed head and the current ArcFace head, labels
  None (plain cosine logits), softmax[:, 1] as the score (:725-730).

Deviations (both where the script cannot do what it intends under torch 2.x):

* the averaged copy of ``embed_head`` is made after its LazyLinear is materialised
  (``feat_dim`` = face_dim + au_dim); the script averages an unmaterialised copy, whose first
  ``update_parameters`` cannot copy into an uninitialised parameter;
* "did the optimizer step" (:688-693) is read from the GradScaler (a skipped step halves the
  scale); the script reads ``optimizer._step_count``, which torch 2.x optimizers no longer
  carry (it was set by the old LR-scheduler step wrapper), so as written the scheduler and the
  averaged models would never advance.
"""
import math

import torch
import torch.nn as nn
import torch.nn.functional as F
from torch.optim.swa_utils import AveragedModel

from .heads import ArcFaceHead, CBFocalLoss


def unpack_batch(batch):
    """(videos, aus, labels) or (videos, aus, labels, au_mask, au_weight) (train_au_face.py:509-518)."""
    if len(batch) == 5:
        return batch
    if len(batch) == 3:
        videos, au_patches, labels = batch
        return videos, au_patches, labels, None, None
    raise RuntimeError(f"Unexpected batch of length {len(batch)}")


def auface_losses(logits_arc, labels, v_tokens, au_tokens, cbfocal, lambda_align=0.2, lambda_temp=0.1):
    """train_au_face.py:666-674 -> (loss, loss_cls, loss_align, loss_temp)."""
    v_pool, au_pool = v_tokens.mean(1), au_tokens.mean(1)
    loss_cls = cbfocal(logits_arc, labels)
    loss_align = F.mse_loss(v_pool, au_pool)
    zero = v_tokens.new_tensor(0.0)
    loss_temp_v = (v_tokens[:, 1:] - v_tokens[:, :-1]).pow(2).mean() if v_tokens.size(1) > 1 else zero
    loss_temp_au = (au_tokens[:, 1:] - au_tokens[:, :-1]).pow(2).mean() if au_tokens.size(1) > 1 else zero
    loss_temp = 0.5 * (loss_temp_v + loss_temp_au)
    return loss_cls + lambda_align * loss_align + lambda_temp * loss_temp, loss_cls, loss_align, loss_temp


class AUFaceTrainer:
    def __init__(self, model, samples_per_cls=(1, 1), feat_dim=1024, lr=1e-4, weight_decay=0.01, max_lr=1e-3,
                 epochs=100, steps_per_epoch=1, accum_steps=4, grad_clip=1.0, lambda_align=0.2, lambda_temp=0.1,
                 use_amp=True, average=True, flat_grads=True, init_scale=2.0 ** 16):
        self.model = model
        dev = next(model.parameters()).device
        self.device = dev
        self.embed_head = nn.Sequential(nn.LazyLinear(256), nn.ReLU(inplace=True), nn.Dropout(0.2),
                                        nn.Linear(256, 128)).to(dev)
        with torch.no_grad():
            self.embed_head(torch.zeros(2, feat_dim, device=dev))   # materialise the LazyLinear
        self.arcface = ArcFaceHead(feat_dim=128, num_classes=2, s=30.0, m=0.30).to(dev)
        self.cbfocal = CBFocalLoss(samples_per_cls=list(samples_per_cls), beta=0.9999, gamma=2.0).to(dev)
        self.ema_model = AveragedModel(model).to(dev) if average else None
        self.ema_embed = AveragedModel(self.embed_head).to(dev) if average else None
        self.params = list(model.parameters()) + list(self.embed_head.parameters()) + list(self.arcface.parameters())
        # flat_grads: gradients in one flat fp32 buffer (xcp.ddp.GradBuckets; the backbones add theirs
        # into it directly), all-reduced across ranks on the micro-batch that steps (DDP no_sync)
        self.buckets = None
        if flat_grads and dev.type == "cuda":
            from .ddp import GradBuckets
            self.buckets = GradBuckets(self.params, module=model)
        self.optimizer = torch.optim.AdamW(self.params, lr=lr, weight_decay=weight_decay)
        self.scheduler = torch.optim.lr_scheduler.OneCycleLR(
            self.optimizer, max_lr=max_lr, epochs=epochs,
            steps_per_epoch=max(1, math.ceil(steps_per_epoch / max(1, accum_steps))), pct_start=0.3)
        self.scaler = torch.amp.GradScaler(init_scale=init_scale, enabled=use_amp and dev.type == "cuda")
        self.use_amp = use_amp
        self.accum_steps, self.grad_clip = accum_steps, grad_clip
        self.lambda_align, self.lambda_temp = lambda_align, lambda_temp
        self._zero_grad()
        self.optimizer_steps = 0

    def _zero_grad(self):
        if self.buckets is not None:
            self.buckets.zero()   # gradients live in the buckets' flat buffer
        else:
            self.optimizer.zero_grad(set_to_none=True)

    def train(self):
        self.model.train()
        self.embed_head.train()
        self.arcface.train()

    def micro_step(self, i, n_batches, batch):
        """One micro-batch of train_au_face.py:639-698; steps the optimizer on every
        ``accum_steps``-th batch (and the last).  Returns (loss tensor, logits_arc, probs)."""
        videos, au_patches, labels, au_mask, au_weight = unpack_batch(batch)
        if videos.dim() == 5 and videos.size(1) != 3 and videos.size(2) == 3:
            videos = videos.permute(0, 2, 1, 3, 4).contiguous()
        dev = self.device
        videos = videos.to(dev, non_blocking=True)
        au_patches = au_patches.to(dev, non_blocking=True)
        labels = labels.long().to(dev, non_blocking=True)
        if au_mask is not None:
            au_mask = au_mask.to(dev, non_blocking=True).float()
        if au_weight is not None:
            au_weight = au_weight.to(dev, non_blocking=True).float()
        step = (i + 1) % self.accum_steps == 0 or (i + 1) == n_batches
        if self.buckets is not None:   # all-reduce only on the micro-batch that steps (DDP no_sync)
            self.buckets.sync = step
        with torch.autocast(device_type="cuda", enabled=dev.type == "cuda" and self.use_amp):
            _, v_tokens, au_tokens = self.model(videos, au_patches, au_mask=au_mask, au_weight=au_weight)
            pooled = torch.cat([v_tokens.mean(1), au_tokens.mean(1)], dim=1)
            embed = self.embed_head(pooled)
            logits_arc = self.arcface(embed, labels)
            loss, _, _, _ = auface_losses(logits_arc, labels, v_tokens, au_tokens, self.cbfocal, self.lambda_align,
                                          self.lambda_temp)
        self.scaler.scale(loss).backward()
        if step:
            if self.buckets is not None:
                self.buckets.allreduce()
            self.scaler.unscale_(self.optimizer)
            torch.nn.utils.clip_grad_norm_(self.params, self.grad_clip)
            scale = self.scaler.get_scale() if self.scaler.is_enabled() else None
            self.scaler.step(self.optimizer)
            self.scaler.update()
            self._zero_grad()
            # the optimizer really stepped (GradScaler skips a step with inf/NaN gradients and
            # halves its scale) -> scheduler and averaged models advance (see module docstring)
            if scale is None or self.scaler.get_scale() >= scale:
                self.optimizer_steps += 1
                self.scheduler.step()
                if self.ema_model is not None:
                    self.ema_model.update_parameters(self.model)
                    self.ema_embed.update_parameters(self.embed_head)
        probs = torch.softmax(logits_arc.detach(), dim=1)[:, 1].float()
        return loss.detach(), logits_arc.detach(), probs

    @torch.no_grad()
    def eval_scores(self, batch):
        """train_au_face.py:711-730: averaged model + averaged embed head, current ArcFace head
        with labels None -> softmax[:, 1]."""
        videos, au_patches, labels, au_mask, au_weight = unpack_batch(batch)
        if videos.dim() == 5 and videos.size(1) != 3 and videos.size(2) == 3:
            videos = videos.permute(0, 2, 1, 3, 4).contiguous()
        model = self.ema_model if self.ema_model is not None else self.model
        embed_head = self.ema_embed if self.ema_embed is not None else self.embed_head
        model.eval()
        embed_head.eval()
        self.arcface.eval()
        dev = self.device
        _, v_tokens, au_tokens = model(videos.to(dev), au_patches.to(dev),
                                       au_mask=None if au_mask is None else au_mask.to(dev).float(),
                                       au_weight=None if au_weight is None else au_weight.to(dev).float())
        embed = embed_head(torch.cat([v_tokens.mean(1), au_tokens.mean(1)], dim=1))
        return torch.softmax(self.arcface(embed), dim=1)[:, 1].float()

    def state_dict(self, best_auc=0.0):
        """The checkpoint train_au_face.py:751-756 saves."""
        model = self.ema_model if self.ema_model is not None else self.model
        embed = self.ema_embed if self.ema_embed is not None else self.embed_head
        return {"model": model.state_dict(), "embed": embed.state_dict(),
                "arcface": self.arcface.state_dict(), "best_auc": best_auc}
