"""Face + action-unit fusion detector for the train_au_face.py harness (BUILD-DEFINED).

The reference imports ``Models.AUFaceModel.AUFaceCrossDetector`` (train_au_face.py:409,
:594; test_au_face.py:13, :285) but the module is not in the snapshot, so its
architecture is unknown.  This build defines one with the call contract the scripts use:

    model = AUFaceCrossDetector(num_aus=17, face_dim=512, au_dim=512, lstm_hidden=256)
    logits, v_tokens, au_tokens = model(videos, au_patches, au_mask=None, au_weight=None)

* ``videos``: [B, 3, T, H, W] (the layout train_au_face.py:643-644 and test_au_face.py:161-162
  normalise every batch to); ``au_patches``: [B, A, 3, h, w] (A <= num_aus AU crops per clip);
  ``au_mask`` [B, A] (> 0: present), ``au_weight`` [B, A] per-AU confidence.
* ``v_tokens`` [B, T, face_dim]: per-frame face tokens, ``au_tokens`` [B, A, au_dim]: per-AU
  tokens (the harness pools both, train_au_face.py:659-661, and regularises their agreement
  and temporal smoothness, :669-672); ``logits`` [B, 2].

Architecture: two Xception backbones (face frames, AU crops) on the xcp engine -- the hot
path; everything after them is a few small GEMMs on PyTorch-ROCm:
  face: Xception(frame) -> Linear(2048, face_dim)                     -> v_tokens
  AU:   Xception(crop)  -> Linear(2048, au_dim) + AU-identity embedding, x au_weight -> au_tokens
  cross: multi-head attention, face tokens query the AU tokens (AUs with mask <= 0 ignored)
  temporal: LSTM(face_dim, lstm_hidden) over v_tokens + cross output; last step
  logits = Linear(lstm_hidden + face_dim, 2)([h_T, mean_t cross])
"""
import torch
import torch.nn as nn

from xcp.lstm import LSTM

from .Xception import xception


class AUFaceCrossDetector(nn.Module):
    def __init__(self, num_aus=17, face_dim=512, au_dim=512, lstm_hidden=256, num_heads=8, pretrained=False):
        super().__init__()
        self.num_aus = num_aus
        self.face_backbone = xception(pretrained=pretrained)
        self.face_backbone.fc = nn.Identity()
        self.au_backbone = xception(pretrained=pretrained)
        self.au_backbone.fc = nn.Identity()
        self.face_proj = nn.Linear(2048, face_dim)
        self.au_proj = nn.Linear(2048, au_dim)
        self.au_embed = nn.Parameter(torch.zeros(num_aus, au_dim))
        nn.init.normal_(self.au_embed, std=0.02)
        self.cross = nn.MultiheadAttention(face_dim, num_heads, kdim=au_dim, vdim=au_dim, batch_first=True)
        self.temporal = LSTM(input_size=face_dim, hidden_size=lstm_hidden, num_layers=1, batch_first=True)
        self.classifier = nn.Linear(lstm_hidden + face_dim, 2)

    @staticmethod
    def frames_first(videos):
        """[B, 3, T, H, W] -> [B, T, 3, H, W]."""
        if videos.dim() != 5 or videos.size(1) != 3:
            raise ValueError(f"videos must be [B, 3, T, H, W], got {tuple(videos.shape)}")
        return videos.permute(0, 2, 1, 3, 4)

    def face_tokens(self, videos):
        v = self.frames_first(videos)
        B, T = v.shape[:2]
        f = self.face_backbone(v.reshape(B * T, *v.shape[2:]))
        return self.face_proj(f).view(B, T, -1)

    def au_tokens(self, au_patches, au_weight=None):
        B, A = au_patches.shape[:2]
        if A > self.num_aus:
            raise ValueError(f"{A} AU patches > num_aus={self.num_aus}")
        a = self.au_backbone(au_patches.reshape(B * A, *au_patches.shape[2:]))
        t = self.au_proj(a).view(B, A, -1) + self.au_embed[:A]
        if au_weight is not None:
            t = t * au_weight.to(t.dtype).unsqueeze(-1)
        return t

    def forward(self, videos, au_patches, au_mask=None, au_weight=None):
        v_tokens = self.face_tokens(videos)
        au_tokens = self.au_tokens(au_patches, au_weight)
        kpm = None
        if au_mask is not None:
            kpm = au_mask <= 0
            kpm = kpm & ~kpm.all(dim=1, keepdim=True)   # a clip without any AU attends to all of them
        fused, _ = self.cross(v_tokens, au_tokens, au_tokens, key_padding_mask=kpm, need_weights=False)
        h = self.temporal(v_tokens + fused)[0][:, -1]
        logits = self.classifier(torch.cat([h, fused.mean(1)], dim=1))
        return logits, v_tokens, au_tokens
