"""Input formats: .flo reader/writer against bytes written by the reference
utils/flowlib.py (tests/golden/formats.npz), the FC2 dataset host logic on a synthetic directory,
and (GPU) the FC2 unpack / uint8-image kernels bit-exact against the oracle restatement of
fc2_dataset.py's ToTensor + Normalize(0.5, 0.5) conversion."""
import os

import numpy as np
import pytest
import torch

from oracle import formats_ref, prng


def test_flo_read_write_match_reference_bytes(golden, tmp_path):
    from gbvst import fc2
    g = golden("formats")
    p = tmp_path / "ref.flo"
    p.write_bytes(g["flo_bytes"].tobytes())
    np.testing.assert_array_equal(fc2.read_flo(str(p)), g["flo_read"])
    q = tmp_path / "ours.flo"
    fc2.write_flo(str(q), g["flo_flow"])
    assert q.read_bytes() == g["flo_bytes"].tobytes()
    bad = tmp_path / "bad.flo"
    bad.write_bytes(b"XXXX" + g["flo_bytes"].tobytes()[4:])
    with pytest.raises(Exception, match="PIEH"):
        fc2.read_flo(str(bad))
    short = tmp_path / "short.flo"
    short.write_bytes(g["flo_bytes"].tobytes()[:-8])
    with pytest.raises(Exception, match="truncated"):
        fc2.read_flo(str(short))


def _fc2_dir(root, n=5, H=12, W=16):
    """Synthetic FC2 layout: data_dir/<frame>.npy ([1,H,W,9]) + style_dir/<style>/<frame>.png."""
    from PIL import Image
    data, style = root / "DATAFiles", root / "styled-files"
    (style / "style1").mkdir(parents=True)
    (style / "style2").mkdir()
    data.mkdir()
    for i in range(n):
        raw = prng.uniform_f32(950 + i, (1, H, W, 9))
        raw[..., 7:9] = prng.normal(960 + i, (1, H, W, 2), std=3.0)
        raw[..., 6] = (raw[..., 6] > 0.3).astype(np.float32)
        raw[0, 0, 0, :6] = [0.0, 1.0, 1.0 / 255, 254.5 / 255, 0.5, 0.99999]
        np.save(data / ("%05d.npy" % i), raw)
        img = (prng.uniform_f32(970 + i, (H, W, 3)) * 255).astype(np.uint8)
        Image.fromarray(img).save(style / "style1" / ("%05d.png" % i))
    return str(data) + "/", str(style) + "/"


def test_fc2_dataset_host_logic(tmp_path):
    from gbvst import fc2
    d, s = _fc2_dir(tmp_path)
    ds = fc2.DatasetFC2(d, s)
    assert len(ds) == 5 and ds.idx2attr == {0: "style1"}
    names = sorted(x[0] for x in ds.dataset)
    assert names == ["%05d.png" % i for i in range(5)]
    for fn, sid, lbl in ds.dataset:
        assert sid == "style1/" + fn and lbl == [False, True]
    raw, sty, lbl = ds[0]
    assert raw.shape == (12, 16, 9) and raw.dtype == np.float32
    assert sty.shape == (12, 16, 3) and sty.dtype == np.uint8
    # the order is the reference's random.seed(1234) shuffle of os.listdir order — deterministic
    assert [x[0] for x in fc2.DatasetFC2(d, s).dataset] == [x[0] for x in ds.dataset]


@pytest.mark.gpu
def test_fc2_unpack_bit_exact(tmp_path):
    import gbvst
    from gbvst import fc2, ops
    gbvst._lib.load()
    d, s = _fc2_dir(tmp_path)
    ds = fc2.DatasetFC2(d, s)
    loader = fc2.FC2Loader(ds, batch_size=2, shuffle=False, device="cuda")
    seen = 0
    for b, (img1, img2, simg, mask, flow) in enumerate(loader):
        ids = list(range(2 * b, min(2 * b + 2, 5)))
        for k, i in enumerate(ids):
            raw, sty, _ = ds[i]
            r1, r2, rm, rf = formats_ref.fc2_sample(raw)
            for got, ref in ((img1, r1), (img2, r2)):
                g = got[k].cpu()
                assert torch.equal(g[..., :3].permute(2, 0, 1), ref)
                assert bool((g[..., 3] == 0).all())
            assert torch.equal(mask[k].cpu(), rm)
            assert torch.equal(flow[k].cpu(), rf)
            assert torch.equal(simg[k].cpu()[..., :3].permute(2, 0, 1), formats_ref.u8_image(sty))
            seen += 1
    assert seen == 5
    # every uint8 level through the image kernel
    lv = torch.arange(256, dtype=torch.uint8).repeat_interleave(3).reshape(1, 16, 16, 3)
    got = ops.u8_image_to_nhwc4(lv.cuda()).cpu()[0, ..., :3].permute(2, 0, 1)
    assert torch.equal(got, formats_ref.u8_image(lv[0].numpy()))
    with pytest.raises(RuntimeError):
        ops.u8_image_to_nhwc4(lv)
