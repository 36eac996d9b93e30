"""Visual clip model (XceptionLSTMV.py:9-70): frozen Xception per frame -> LSTM -> FC head.

Same constructor, submodules (``feature_extractor``, ``lstm``, ``fc_layers``,
``fc_out``, ``sigmoid``), init order and state_dict as the reference.  The
backbone runs on the xcp engine (one pass over the B*T frame batch, temporal
batching as XceptionLSTMV.py:55), ``lstm`` is the fused-kernel ``nn.LSTM``
drop-in; the small FC head stays on PyTorch-ROCm (hipBLASLt).

``pretrained`` defaults to True as in the reference (XceptionLSTMV.py:12); offline
that needs a local weight file (see ``Models.Xception.xception``).
"""
import torch
import torch.nn as nn

from xcp.lstm import LSTM

from .Xception import xception


class XceptionLSTMV(nn.Module):
    def __init__(self, hidden_dim, pretrained=True):
        super(XceptionLSTMV, self).__init__()
        self.feature_extractor = xception(pretrained=pretrained)
        self.feature_extractor.fc = nn.Identity()
        for param in self.feature_extractor.parameters():
            param.requires_grad = False
        self.lstm = LSTM(input_size=2048, hidden_size=hidden_dim, num_layers=1, batch_first=True)
        self.fc_layers = nn.Sequential(
            nn.Linear(hidden_dim, 1024), nn.ReLU(), nn.Dropout(0.3),
            nn.Linear(1024, 1024), nn.ReLU(), nn.Dropout(0.3),
            nn.Linear(1024, 1024), nn.ReLU(), nn.Dropout(0.3),
            nn.Linear(1024, 1024), nn.ReLU(), nn.Dropout(0.3),
        )
        self.fc_out = nn.Linear(1024, 1)
        self.sigmoid = nn.Sigmoid()

    def extract_features(self, video_batch, device=None):
        """[B,T,3,H,W] -> [B,T,2048] (XceptionLSTMV.py:46-63).  ``device`` may also be the
        ``seq_lengths`` tensor the active train_visual.py:568 passes; it is ignored
        there, as the shipped model ignores sequence lengths."""
        if device is not None and not torch.is_tensor(device):
            self.feature_extractor.to(device)
        batch_size, seq_len, c, h, w = video_batch.shape
        frames = video_batch.reshape(batch_size * seq_len, c, h, w)
        frame_features = self.feature_extractor(frames)
        return frame_features.view(batch_size, seq_len, -1)

    def forward(self, features):
        lstm_out, _ = self.lstm(features)
        lstm_out = lstm_out[:, -1, :]
        dense_out = self.fc_layers(lstm_out)
        return self.sigmoid(self.fc_out(dense_out))
