"""Face-clip dataset (reference: video_dataloader.py:6-68).

Same interface and semantics: ``.npy`` files of uint8 frames ``[T, H, W, 3]``, label
from the file-name prefix (``real_`` -> 0, anything else -> 1), frames converted to
fp32 in [0, 1] and permuted to ``[T, 3, H, W]`` (no mean/std normalisation, as the
reference), ``collate_fn`` zero-pads the time axis to the batch maximum.

Differences, all compatible: the padded frame size is taken from the data instead of
the hard-coded 256x256 of video_dataloader.py:61 (which raises on any other size);
file order is sorted (``os.listdir`` order is filesystem-dependent);
``clips_to_device`` moves a collated batch to the GPU, optionally as bf16.
"""
import os

import numpy as np
import torch
from torch.utils.data import DataLoader, Dataset


def label_from_name(path):
    return 0 if os.path.basename(path).split("_")[0].lower() == "real" else 1


class FaceDataset(Dataset):
    def __init__(self, folder_path):
        self.folder_path = folder_path
        self.npy_files = sorted(os.path.join(folder_path, f) for f in os.listdir(folder_path) if f.endswith(".npy"))

    def __len__(self):
        return len(self.npy_files)

    def __getitem__(self, idx):
        npy_file = self.npy_files[idx]
        face_data = np.load(npy_file, allow_pickle=False)   # (num_frames, H, W, 3) uint8
        label = label_from_name(npy_file)
        face_data = torch.from_numpy(np.ascontiguousarray(face_data)).to(torch.float32).permute(0, 3, 1, 2) / 255.0
        return face_data, torch.tensor([label], dtype=torch.float32)


def collate_fn(batch):
    videos, labels = zip(*batch)
    max_seq_len = max(v.size(0) for v in videos)
    c, h, w = videos[0].shape[1:]
    padded = torch.zeros((len(videos), max_seq_len, c, h, w), dtype=torch.float32)
    for i, v in enumerate(videos):
        padded[i, :v.size(0)] = v
    return padded, torch.stack(labels)


def get_face_dataloader(folder_path, batch_size=1, shuffle=False, num_workers=0):
    dataset = FaceDataset(folder_path)
    return DataLoader(dataset, batch_size=batch_size, shuffle=shuffle, pin_memory=torch.cuda.is_available(),
                      collate_fn=collate_fn, num_workers=num_workers)


def clips_to_device(batch, device, dtype=torch.float32, non_blocking=True):
    clips, labels = batch
    return clips.to(device, non_blocking=non_blocking).to(dtype), labels.to(device, non_blocking=non_blocking)
