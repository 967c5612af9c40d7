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


# --------------------------------------------------------------- StarGAN FC2 7-tuple (C4)
class _AttrDict(dict):
    """munch.Munch stand-in (attribute access to a dict; munch is not installed)."""

    def __getattr__(self, k):
        try:
            return self[k]
        except KeyError as e:
            raise AttributeError(k) from e


class StarGANDatasetFC2(torch.utils.data.Dataset):
    """methods/GAN-based/StarGAN/sg2_core/data_loader.py:217-293 DatasetFC2: for every source image
    and style pair (src, ref) in {(0, 0)} + {(0, i), (i, 0), (i, i)} for styles i = 1..num_dom-1, the
    7-tuple (src_img, src_img2, src_lbl, ref_img, ref_lbl, mask, flow): the source frame in style
    src_lbl (style_dir), its second frame (temp_dir, '<name>_2.jpg'), the reference frame in style
    ref_lbl, and mask / flow from the FC2 .npy block (channels 6:7 / 7:9, moved to CHW).  Paths are
    joined by string concatenation as the reference does (directories end with '/').  The list is
    shuffled once with random.seed(1234) (:291-292); base_len: the per-style image count the
    reference asserts (22208 for FC2; None skips the check)."""

    def __init__(self, data_dir, style_dir, temp_dir, transform=None, num_dom=4, base_len=22208):
        from .sintel_eval import sintel_transform
        self.data_dir, self.style_dir, self.temp_dir = data_dir, style_dir, temp_dir
        self.transform = transform or sintel_transform
        self.num_dom, self.base_len = num_dom, base_len
        self.dataset, self.styles = [], []
        self.preprocess()
        self.num_images = len(self.dataset)

    def preprocess(self):
        style_list = sorted(os.listdir(self.style_dir))[:self.num_dom]
        for sty in style_list:
            n = len(os.listdir(self.style_dir + sty))
            if self.base_len is not None:
                assert self.base_len == n, (self.base_len, n)
            self.styles.append(sty)
        for img in sorted(os.listdir(self.style_dir + style_list[0])):
            file = "/" + img
            self.dataset.append([file, 0, 0])
            for i in range(len(style_list) - 1):
                self.dataset.append([file, 0, i + 1])
                self.dataset.append([file, i + 1, 0])
                self.dataset.append([file, i + 1, i + 1])
        random.seed(1234)
        random.shuffle(self.dataset)

    def __getitem__(self, index):
        from PIL import Image
        file, src_lbl, ref_lbl = self.dataset[index]
        src_img = self.transform(Image.open(self.style_dir + self.styles[src_lbl] + file))
        src_img2 = self.transform(Image.open(self.temp_dir + self.styles[src_lbl] + file[:-4] + "_2.jpg"))
        ref_img = self.transform(Image.open(self.style_dir + self.styles[ref_lbl] + file))
        np_data = np.load(self.data_dir + file[:-4] + ".npy", allow_pickle=False)[0]
        mask = torch.from_numpy(np.ascontiguousarray(np.moveaxis(np_data[:, :, 6:7], 2, 0)))
        flow = torch.from_numpy(np.ascontiguousarray(np.moveaxis(np_data[:, :, 7:9], 2, 0)))
        return (src_img, src_img2, torch.tensor(src_lbl, dtype=torch.long), ref_img,
                torch.tensor(ref_lbl, dtype=torch.long), mask, flow)

    def __len__(self):
        return self.num_images


def get_loaderFC2(data_dir, style_dir, temp_dir, batch_size=4, num_workers=0, num_dom=2, mode="train",
                  base_len=22208):
    """sg2_core/data_loader.py:295-317: ToTensor + Normalize(0.5) transform, 97 % / 3 % random split,
    shuffling DataLoaders; returns (train_loader, eval_loader)."""
    full = StarGANDatasetFC2(data_dir, style_dir, temp_dir, None, num_dom, base_len)
    train_size = int(0.97 * len(full))
    train_ds, eval_ds = torch.utils.data.random_split(full, [train_size, len(full) - train_size])
    mk = lambda ds: torch.utils.data.DataLoader(ds, batch_size=batch_size, shuffle=True,  # noqa: E731
                                                num_workers=num_workers)
    return mk(train_ds), mk(eval_ds)


class FC2Fetcher:
    """sg2_core/data_loader.py:321-348: endless iterator over an FC2 loader; each item is the 7-tuple
    plus latent codes z_trg, z_trg2 ~ N(0, 1) [B, latent_dim], all on the device, as an attribute dict
    (x_src, x2_src, y_src, x_ref, y_ref, mask, flow, z_trg, z_trg2)."""

    def __init__(self, loader, loader_ref=None, latent_dim=16, mode='', device=None):
        self.loader, self.latent_dim, self.mode = loader, latent_dim, mode
        self.device = device or torch.device('cuda' if torch.cuda.is_available() else 'cpu')
        self.iter = None

    def _fetch_inputs_fc2(self):
        try:
            if self.iter is None:
                raise StopIteration
            return next(self.iter)
        except StopIteration:
            self.iter = iter(self.loader)
            return next(self.iter)

    def __iter__(self):
        return self

    def __next__(self):
        src_img, src_img2, src_lbl, ref_img, ref_lbl, mask, flow = self._fetch_inputs_fc2()
        z_trg = torch.randn(src_img.size(0), self.latent_dim)
        z_trg2 = torch.randn(src_img.size(0), self.latent_dim)
        inputs = dict(x_src=src_img, x2_src=src_img2, y_src=src_lbl, x_ref=ref_img, y_ref=ref_lbl,
                      mask=mask, flow=flow, z_trg=z_trg, z_trg2=z_trg2)
        return _AttrDict({k: v.to(self.device) for k, v in inputs.items()})
