"""FC2 and .flo input formats (SURVEY §8f "formats") feeding the CycleGANCon step.

Mirrors methods/GAN-based/CycleGANCon/fc2_dataset.py (``DatasetFC2``, ``FC2_DatasetDataLoader``) and
utils/flowlib.py (``readFlow`` / ``writeFlow``).  Host side only reads files; the per-pixel work —
uint8 round trip + ToTensor + Normalize(0.5, 0.5) of both frames, mask and flow de-interleave — is
one device kernel (``vst_fc2_unpack``) over the raw [B,H,W,9] block, producing the NHWC4 / planar
tensors ``CycleGANModel.set_input_nhwc`` takes.  Batches are staged through pinned host memory and
copied on a side stream one batch ahead of the consumer.
"""
import os
import random

import numpy as np
import torch

from . import ops

PIEH = b"PIEH"


# ----------------------------------------------------------------------------------- .flo
def read_flo(path):
    """utils/flowlib.py:33-50 readFlow: 'PIEH', int32 W, int32 H, float32 [H][W][2]."""
    with open(path, "rb") as f:
        if f.read(4) != PIEH:
            raise Exception("Flow file header does not contain PIEH")
        w = int(np.fromfile(f, np.int32, 1)[0])
        h = int(np.fromfile(f, np.int32, 1)[0])
        flow = np.fromfile(f, np.float32, w * h * 2)
    if flow.size != w * h * 2:
        raise Exception("Flow file %s is truncated" % path)
    return flow.reshape(h, w, 2)


def write_flo(path, flow):
    """utils/flowlib.py:52-58 writeFlow."""
    flow = np.asarray(flow)
    with open(path, "wb") as f:
        f.write(PIEH)
        np.array([flow.shape[1], flow.shape[0]], dtype=np.int32).tofile(f)
        flow.astype(np.float32).tofile(f)


# ------------------------------------------------------------------------------------ FC2
class DatasetFC2:
    """fc2_dataset.py:19-72: samples are (npy block of a frame pair, one styled frame, label).
    ``__getitem__`` returns host arrays (raw float32 [H,W,9], style uint8 [H,W,3], label list)."""

    def __init__(self, data_dir, style_dir):
        self.data_dir, self.style_dir = data_dir, style_dir
        self.dataset, self.attr2idx, self.idx2attr = [], {}, {}
        self.preprocess()
        self.num_images = len(self.dataset)

    def preprocess(self):
        names = sorted(os.listdir(self.style_dir))[:1]
        for i, attr in enumerate(names):
            self.attr2idx[attr], self.idx2attr[i] = i, attr
            for filename in os.listdir(os.path.join(self.style_dir, attr)):
                label = [attr == sub for sub in ["style0"] + names]
                self.dataset.append([filename, attr + "/" + filename, label])
        random.seed(1234)
        random.shuffle(self.dataset)

    def __len__(self):
        return self.num_images

    def __getitem__(self, index):
        from PIL import Image
        img_id, simg_id, slbl = self.dataset[index]
        raw = np.load(self.data_dir + img_id[:-4] + ".npy", allow_pickle=False)[0]
        simg = np.asarray(Image.open(os.path.join(self.style_dir, simg_id)).convert("RGB"), dtype=np.uint8)
        return np.ascontiguousarray(raw, dtype=np.float32), np.ascontiguousarray(simg), slbl


class FC2Loader:
    """FC2_DatasetDataLoader (fc2_dataset.py:74-111) for the device path: yields
    (real_A, real_A2, real_B, mask, flow) ready for ``CycleGANModel.set_input_nhwc``; batch_size,
    serial_batches (no shuffle), max_dataset_size as in the reference options."""

    def __init__(self, dataset, batch_size=1, shuffle=True, max_dataset_size=float("inf"), device="cuda",
                 seed=0, drop_last=False):
        self.dataset, self.batch_size, self.shuffle = dataset, batch_size, shuffle
        self.max_dataset_size, self.device = max_dataset_size, torch.device(device)
        self.rng = np.random.default_rng(seed)
        self.drop_last = drop_last
        self._stream = None

    def __len__(self):
        return int(min(len(self.dataset), self.max_dataset_size))

    def _batches(self):
        idx = self.rng.permutation(len(self.dataset)) if self.shuffle else np.arange(len(self.dataset))
        for i in range(0, len(idx), self.batch_size):
            if i >= self.max_dataset_size:
                break
            b = idx[i:i + self.batch_size]
            if self.drop_last and len(b) < self.batch_size:
                break
            yield b

    def _stage(self, ids):
        items = [self.dataset[int(i)] for i in ids]
        raw = torch.from_numpy(np.stack([it[0] for it in items])).pin_memory()
        sty = torch.from_numpy(np.stack([it[1] for it in items])).pin_memory()
        if self._stream is None:
            self._stream = torch.cuda.Stream(device=self.device)
        with torch.cuda.stream(self._stream):
            raw_d = raw.to(self.device, non_blocking=True)
            sty_d = sty.to(self.device, non_blocking=True)
            out = self.unpack(raw_d, sty_d)
            ev = torch.cuda.Event()
            ev.record(self._stream)
        return out, ev, (raw, sty)

    @staticmethod
    def unpack(raw_d, sty_d):
        img1, img2, mask, flow = ops.fc2_unpack(raw_d)
        return img1, img2, ops.u8_image_to_nhwc4(sty_d), mask, flow

    def __iter__(self):
        pending = None
        for ids in self._batches():
            nxt = self._stage(ids)
            if pending is not None:
                yield self._finish(pending)
            pending = nxt
        if pending is not None:
            yield self._finish(pending)

    @staticmethod
    def _finish(pending):
        out, ev, _host = pending
        cur = torch.cuda.current_stream()
        cur.wait_event(ev)
        for t in out:  # allocated on the copy stream, consumed on this one
            t.record_stream(cur)
        return out
