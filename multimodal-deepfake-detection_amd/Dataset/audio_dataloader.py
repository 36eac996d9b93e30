"""MFCC clip dataset (reference: audio_dataloader.py:6-47).

``.npy`` MFCC arrays ``[T, 13]`` (T = 120 in wavfake_audio_dataset.py), label from the
file-name prefix, expanded to ``[T, 3, 13]`` by repeating the coefficient row over 3
channels (audio_dataloader.py:25-26); ``collate_fn`` zero-pads T to the batch maximum
giving ``[B, T, 3, 13]``.  File order is sorted.
"""
import os

import numpy as np
import torch
from torch.utils.data import DataLoader, Dataset


class AudioDataset(Dataset):
    def __init__(self, folder_path):
        self.folder_path = folder_path
        self.npy_files = sorted(os.path.join(folder_path, f) for f in os.listdir(folder_path) if f.endswith(".npy"))

    def __len__(self):
        return len(self.npy_files)

    def __getitem__(self, idx):
        npy_file = self.npy_files[idx]
        mfcc = np.load(npy_file, allow_pickle=False)
        label = 0 if os.path.basename(npy_file).split("_")[0].lower() == "real" else 1
        mfcc = torch.tensor(mfcc, dtype=torch.float32).unsqueeze(1).repeat(1, 3, 1)
        return mfcc, torch.tensor([label], dtype=torch.float32)


def collate_fn(batch):
    mfccs, labels = zip(*batch)
    max_seq_len = max(m.size(0) for m in mfccs)
    padded = torch.zeros((len(mfccs), max_seq_len, 3, mfccs[0].shape[-1]), dtype=torch.float32)
    for i, m in enumerate(mfccs):
        padded[i, :m.size(0)] = m
    return padded, torch.stack(labels)


def get_audio_dataloader(folder_path, batch_size=1, shuffle=False, num_workers=0):
    return DataLoader(AudioDataset(folder_path), batch_size=batch_size, shuffle=shuffle, collate_fn=collate_fn,
                      num_workers=num_workers)
