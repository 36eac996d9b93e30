"""Audio clip model (XceptionLSTMA.py:5-59): MFCC frames resized to 64x64 -> Xception -> LSTM -> FC.

Same module surface as the reference.  ``extract_features`` reshapes
``[B,T,3,13]`` to ``[B*T,3,13,1]``, resizes bilinearly to 64x64
(align_corners=False, XceptionLSTMA.py:46) with the HIP kernel ``xcp_resize_bilinear``
and runs the xcp backbone.
"""
import torch
import torch.nn as nn
from xcp import ops
from xcp.lstm import LSTM

from .Xception import xception


class XceptionLSTMA(nn.Module):
    def __init__(self, hidden_dim, pretrained=True):
        super(XceptionLSTMA, self).__init__()
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

    def extract_features(self, audio_batch, device=None):
        if device is not None and not torch.is_tensor(device):
            self.feature_extractor.to(device)
        batch_size, time_steps, c, n_mfcc = audio_batch.shape
        frames = audio_batch.reshape(batch_size * time_steps, c, n_mfcc, 1)
        frames = ops.resize_bilinear(frames, (64, 64))
        frame_features = self.feature_extractor(frames)
        return frame_features.view(batch_size, time_steps, frame_features.shape[-1])

    def forward(self, features):
        lstm_out, _ = self.lstm(features)
        lstm_out = lstm_out[:, -1, :]
        dense_out = self.fc_layers(lstm_out)
        return self.sigmoid(self.fc_out(dense_out))
