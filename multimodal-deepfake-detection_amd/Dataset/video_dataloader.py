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


# ---- uint8 path: the same clips with the /255 + permute + pad done on the GPU ----------------
# The host ships uint8 [B, Tmax, H, W, 3] (a quarter of the fp32 bytes over PCIe) and
# xcp_frames_u8_to_f32 expands it in HBM, bit-identical to FaceDataset + collate_fn.

class FaceDatasetU8(FaceDataset):
    def __getitem__(self, idx):
        npy_file = self.npy_files[idx]
        face_data = np.load(npy_file, allow_pickle=False)   # (num_frames, H, W, 3) uint8
        if face_data.dtype != np.uint8 or face_data.ndim != 4 or face_data.shape[-1] != 3:
            raise ValueError(f"{npy_file}: expected uint8 [T, H, W, 3] frames")
        label = label_from_name(npy_file)
        return torch.from_numpy(np.ascontiguousarray(face_data)), torch.tensor([label], dtype=torch.float32)


def collate_u8(batch):
    """-> (uint8 [B, Tmax, H, W, 3] zero-padded, labels [B, 1], lengths int32 [B])."""
    videos, labels = zip(*batch)
    lengths = torch.tensor([v.size(0) for v in videos], dtype=torch.int32)
    h, w, c = videos[0].shape[1:]
    padded = torch.zeros((len(videos), int(lengths.max()), h, w, c), dtype=torch.uint8)
    for i, v in enumerate(videos):
        padded[i, :v.size(0)] = v
    return padded, torch.stack(labels), lengths


def get_face_dataloader_u8(folder_path, batch_size=1, shuffle=False, num_workers=0):
    dataset = FaceDatasetU8(folder_path)
    return DataLoader(dataset, batch_size=batch_size, shuffle=shuffle, pin_memory=torch.cuda.is_available(),
                      collate_fn=collate_u8, num_workers=num_workers)


def clips_u8_to_device(batch, device, non_blocking=True):
    """uint8 batch from get_face_dataloader_u8 -> (fp32 [B, Tmax, 3, H, W] clips, labels) on
    the GPU, equal to clips_to_device(collate_fn(...)) of the same files."""
    from xcp import ops
    frames, labels, lengths = batch
    B, T, H, W, _ = frames.shape
    f = frames.to(device, non_blocking=non_blocking)
    ln = lengths.to(device, non_blocking=non_blocking)
    out = torch.empty((B, T, 3, H, W), device=f.device, dtype=torch.float32)
    ops.frames_u8_to_f32(f, ln, out)
    return out, labels.to(device, non_blocking=non_blocking)
