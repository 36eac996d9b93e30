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


class PinnedClipReader:
    """Double-buffered clip reader: the uint8 clips of a folder (FaceDataset's files, order and
    labels) are read on a background thread straight into one of two pinned host buffers,
    copied to the GPU on a side stream, and expanded there by ``xcp_frames_prep`` (x / 255,
    optional bilinear resize, fp32 or bf16, planar or channels_last).  While the model runs on
    batch i, batch i + 1 is read from disk and copied over PCIe.

    Iterating yields ``(clips [B, Tmax, 3, OH, OW], labels [B, 1] fp32, lengths [B] int32)`` on
    the device, clips equal to ``collate_fn`` of FaceDataset items (then resized / cast).
    """

    def __init__(self, folder_path, batch_size, device, size=None, dtype=torch.float32, channels_last=False,
                 shuffle=False, seed=0, drop_last=False):
        self.files = FaceDataset(folder_path).npy_files
        self.batch_size = batch_size
        self.device = torch.device(device)
        self.size, self.dtype, self.channels_last = size, dtype, channels_last
        self.shuffle, self.seed, self.drop_last = shuffle, seed, drop_last
        self.epoch = 0

    def __len__(self):
        n = len(self.files)
        return n // self.batch_size if self.drop_last else -(-n // self.batch_size)

    def batches(self):
        order = np.arange(len(self.files))
        if self.shuffle:
            order = np.random.default_rng(self.seed + self.epoch).permutation(len(self.files))
        bs = self.batch_size
        out = [order[i:i + bs] for i in range(0, len(order), bs)]
        if self.drop_last and out and len(out[-1]) < bs:
            out.pop()
        return [[self.files[j] for j in b] for b in out]

    @staticmethod
    def read_batch(paths, buf=None, pin=False):
        """Host side of one batch: the clips' uint8 frames into ``buf`` (grown / allocated as
        needed, pinned when ``pin``) as [B, Tmax, H, W, 3]; returns (frames view, labels,
        lengths).  Frames past a clip's length are left as they are (the kernel ignores them)."""
        arrs = [np.load(p, mmap_mode="r", allow_pickle=False) for p in paths]
        for p, a in zip(paths, arrs):
            if a.dtype != np.uint8 or a.ndim != 4 or a.shape[-1] != 3:
                raise ValueError(f"{p}: expected uint8 [T, H, W, 3] frames")
        hw = {a.shape[1:] for a in arrs}
        if len(hw) != 1:
            raise ValueError(f"clips of one batch must share the frame size, got {sorted(hw)}")
        (H, W, _), = hw
        lengths = torch.tensor([a.shape[0] for a in arrs], dtype=torch.int32)
        shape = (len(arrs), int(lengths.max()), H, W, 3)
        n = int(np.prod(shape))
        if buf is None or buf.numel() < n:
            buf = torch.empty(max(n, 0 if buf is None else 2 * buf.numel()), dtype=torch.uint8, pin_memory=pin)
        frames = buf[:n].view(shape)
        fn = frames.numpy()
        for i, a in enumerate(arrs):
            fn[i, :a.shape[0]] = a
        labels = torch.tensor([[float(label_from_name(p))] for p in paths], dtype=torch.float32)
        return buf, frames, labels, lengths

    def __iter__(self):
        import queue
        import threading
        from xcp import ops
        batches = self.batches()
        self.epoch += 1
        copy_stream = torch.cuda.Stream(self.device)
        bufs = [None, None]
        free = [threading.Event(), threading.Event()]   # host buffer may be refilled
        for e in free:
            e.set()
        copied = [None, None]                            # device event: H2D copy of the slot done
        q = queue.Queue(maxsize=1)
        stop = threading.Event()

        def reader():
            try:
                for i, paths in enumerate(batches):
                    slot = i & 1
                    while not free[slot].wait(0.1):
                        if stop.is_set():
                            return
                    free[slot].clear()
                    if copied[slot] is not None:
                        copied[slot].synchronize()
                    bufs[slot], frames, labels, lengths = self.read_batch(paths, bufs[slot], pin=True)
                    q.put((slot, frames, labels, lengths))
                q.put(None)
            except BaseException as exc:   # surfaced on the consumer side
                q.put(exc)

        th = threading.Thread(target=reader, daemon=True)
        th.start()
        try:
            while True:
                item = q.get()
                if item is None:
                    break
                if isinstance(item, BaseException):
                    raise item
                slot, frames, labels, lengths = item
                with torch.cuda.stream(copy_stream):
                    f = frames.to(self.device, non_blocking=True)
                    ln = lengths.to(self.device, non_blocking=True)
                    lab = labels.to(self.device, non_blocking=True)
                    ev = torch.cuda.Event()
                    ev.record(copy_stream)
                copied[slot] = ev
                free[slot].set()
                cur = torch.cuda.current_stream(self.device)
                cur.wait_event(ev)
                for t in (f, ln, lab):
                    t.record_stream(cur)
                clips = ops.frames_prep(f, ln, self.size, self.dtype, self.channels_last)
                yield clips, lab, ln
        finally:
            stop.set()
            th.join(timeout=5)


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
