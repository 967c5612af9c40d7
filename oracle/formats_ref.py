"""CPU oracle for the input formats: FC2 sample conversion and .flo files.

TEST INFRASTRUCTURE ONLY (see oracle/__init__.py).
  methods/GAN-based/CycleGANCon/fc2_dataset.py:35-41 + :79-81   DatasetFC2.__getitem__ with
      T.ToTensor() + T.Normalize((0.5,)*3, (0.5,)*3): img = Normalize(ToTensor(uint8(v * 255.0)))
  utils/flowlib.py:33-58                                       readFlow / writeFlow
fc2_dataset.py imports torchvision (absent), so the conversion is restated from torchvision's
published ToTensor (uint8 HWC -> float CHW / 255) and Normalize ((t - mean) / std) semantics:
parity of the FC2 conversion is pinned only by this restatement.  readFlow/writeFlow are pinned by
tests/golden/formats.npz, written by importing the reference utils/flowlib.py
(oracle/gen_golden_formats.py).
"""
import numpy as np
import torch


def fc2_sample(raw):
    """raw float32 [H,W,9] -> (img1 [3,H,W], img2 [3,H,W], mask [1,H,W], flow [2,H,W]) as torch."""
    def img(a):
        u8 = np.uint8(a * 255.0)
        t = torch.from_numpy(np.ascontiguousarray(u8)).permute(2, 0, 1).contiguous().float().div(255)
        return t.sub(0.5).div(0.5)
    mask = torch.from_numpy(np.ascontiguousarray(np.moveaxis(raw[:, :, 6:7], 2, 0)))
    flow = torch.from_numpy(np.ascontiguousarray(np.moveaxis(raw[:, :, 7:9], 2, 0)))
    return img(raw[:, :, :3]), img(raw[:, :, 3:6]), mask, flow


def u8_image(u8):
    """uint8 [H,W,3] -> Normalize(ToTensor(.)) [3,H,W]."""
    return torch.from_numpy(np.ascontiguousarray(u8)).permute(2, 0, 1).contiguous().float().div(255).sub(0.5).div(0.5)
