"""Host side of the Sintel evaluation harness (gbvst.sintel_eval), CPU only: the frame dataset
(methods/GAN-based/CycleGAN/sintel_eval.py:63-103 and the 432-row utils/sintel_eval.py:62-102
variant), the ToTensor + Normalize(0.5) transform (torchvision is absent: restated, checked against
the formula) and the PNG writer (vutils.save_image of denormalize(x): uint8(x*255 + 0.5))."""
import json
import os

import numpy as np
import torch
from PIL import Image


def _frames(d, n=7, H=40, W=48, seed=0):
    os.makedirs(d, exist_ok=True)
    rng = np.random.default_rng(seed)
    arrs = []
    for i in range(n):
        a = rng.integers(0, 256, (H, W, 3), dtype=np.uint8)
        Image.fromarray(a).save(os.path.join(d, "frame_%04d.png" % (i + 1)))
        arrs.append(a)
    return arrs


def test_transform_and_dataset(tmp_path):
    from gbvst import sintel_eval as se
    arrs = _frames(str(tmp_path / "alley_1"))
    ds = se.SingleSintelVideo(str(tmp_path / "alley_1"))
    assert len(ds) == 7
    img, last, past = ds[0]
    ref = (torch.from_numpy(arrs[0]).permute(2, 0, 1).float() / 255 - 0.5) / 0.5
    assert torch.equal(img, ref)
    assert last.dim() == 0 and past.dim() == 0  # placeholders (sintel_eval.py:76-77)
    img, last, past = ds[5]
    assert torch.equal(last, (torch.from_numpy(arrs[4]).permute(2, 0, 1).float() / 255 - 0.5) / 0.5)
    assert torch.equal(past, (torch.from_numpy(arrs[0]).permute(2, 0, 1).float() / 255 - 0.5) / 0.5)
    crop = se.SingleSintelVideo(str(tmp_path / "alley_1"), crop_rows=32)
    a, b, c = crop[6]
    assert a.shape == (3, 32, 48) and b.shape == (3, 32, 48) and c.shape == (3, 32, 48)


def test_save_image_quantisation(tmp_path):
    from gbvst import sintel_eval as se
    x = torch.linspace(-1.2, 1.2, 3 * 8 * 10).view(3, 8, 10)
    f = str(tmp_path / "f.png")
    se.save_image(x, 1, f)
    got = np.asarray(Image.open(f))
    want = (((x + 1) / 2).clamp(0, 1) * 255 + 0.5).clamp(0, 255).permute(1, 2, 0).to(torch.uint8).numpy()
    assert np.array_equal(got, want)


def test_save_dict_as_json(tmp_path):
    from gbvst import sintel_eval as se
    d = {"TCL-ST_a_s1": 1.0, "TCL-ST_a_s2": 2.0, "TCL-ST_a_s3": 3.0,
         "TCL-ST_b_s1": 3.0, "TCL-ST_b_s2": 4.0, "TCL-ST_b_s3": 5.0}
    out = se.save_dict_as_json("TCL-ST", dict(d), str(tmp_path), 4)
    assert abs(out["TCL-ST_mean"] - 3.0) < 1e-12
    assert abs(out["TCL-ST_mean_s1"] - 2.0) < 1e-12 and abs(out["TCL-ST_mean_s3"] - 4.0) < 1e-12
    assert json.load(open(tmp_path / "TCL-ST.json")) == out
