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


def test_stargan_fc2_seven_tuple(tmp_path):
    """StarGAN's FC2 7-tuple loader (sg2_core/data_loader.py:217-348): dataset order (style pairs,
    random.seed(1234) shuffle), the item tuple (frames through ToTensor + Normalize(0.5), labels,
    mask / flow from the .npy block in CHW), the 97/3 split and the fetcher's attribute dict."""
    import random

    import numpy as np
    from PIL import Image

    from gbvst import fc2
    rng = np.random.default_rng(3)
    data, sty, tmp = tmp_path / "npy", tmp_path / "style", tmp_path / "temp"
    H, W, names, styles = 8, 12, ["a.jpg", "b.jpg", "c.jpg"], ["s0", "s1", "s2"]
    os.makedirs(data)
    for n in names:
        np.save(data / (n[:-4] + ".npy"), rng.random((1, H, W, 9)).astype(np.float32))
        for s in styles:
            for d, suffix in ((sty, ""), (tmp, "_2")):
                os.makedirs(d / s, exist_ok=True)
                Image.fromarray(rng.integers(0, 256, (H, W, 3), dtype=np.uint8)).save(d / s / (n[:-4] + suffix + ".jpg"))
    ds = fc2.StarGANDatasetFC2(str(data) + "/", str(sty) + "/", str(tmp) + "/", num_dom=3, base_len=3)
    expect = []
    for n in names:
        expect.append(["/" + n, 0, 0])
        for i in range(2):
            expect += [["/" + n, 0, i + 1], ["/" + n, i + 1, 0], ["/" + n, i + 1, i + 1]]
    random.seed(1234)
    random.shuffle(expect)
    assert ds.dataset == expect and len(ds) == 21
    src, src2, sl, ref, rl, mask, flow = ds[0]
    f, s_l, r_l = expect[0]
    raw = np.load(data / (f[1:-4] + ".npy"))[0]
    assert src.shape == (3, H, W) and src2.shape == (3, H, W) and ref.shape == (3, H, W)
    assert int(sl) == s_l and int(rl) == r_l
    assert np.array_equal(mask.numpy(), np.moveaxis(raw[:, :, 6:7], 2, 0))
    assert np.array_equal(flow.numpy(), np.moveaxis(raw[:, :, 7:9], 2, 0))
    img = np.asarray(Image.open(str(sty) + "/" + styles[s_l] + f).convert("RGB"))
    assert torch.equal(src, (torch.from_numpy(img.copy()).permute(2, 0, 1).float() / 255 - 0.5) / 0.5)
    tr, ev = fc2.get_loaderFC2(str(data) + "/", str(sty) + "/", str(tmp) + "/", batch_size=2, num_dom=3, base_len=3)
    assert len(tr.dataset) == int(0.97 * 21) and len(ev.dataset) == 21 - int(0.97 * 21)
    batch = next(fc2.FC2Fetcher(tr, latent_dim=16, device=torch.device("cpu")))
    assert batch.x_src.shape == (2, 3, H, W) and batch.z_trg.shape == (2, 16) and batch.flow.shape == (2, 2, H, W)
