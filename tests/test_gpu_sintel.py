"""End-to-end Sintel evaluation harness on the GPU (gbvst.sintel_eval.evaluate_sintel, the
methods/GAN-based/CycleGAN/sintel_eval.py:143-235 driver) over a synthetic Sintel tree: two videos
(training/final and test/final), a checkpoint directory loaded through create_model + setup, PNG
frames written per video, TCL-ST / TCL-LT / DT JSONs.  The TCL values are checked against the CPU
oracle (oracle/cpu_ref.py: the reference generator, warp, fbcCheckTorch and TCL formula) run on the
same decoded frames with the same flows; the flow source is a deterministic elementwise function of
the two frames (RAFT's pretrained weights are not available; RAFT itself is tested in
test_gpu_raft.py), evaluated identically on both sides."""
import json
import os

import numpy as np
import pytest
import torch
from PIL import Image

pytestmark = pytest.mark.gpu


def _flow(a, b):
    return (torch.stack([a[:, 0] - b[:, 1], a[:, 2] - b[:, 0]], 1) * 2.0).contiguous()


def _write_video(d, n, H, W, seed):
    os.makedirs(d, exist_ok=True)
    rng = np.random.default_rng(seed)
    base = rng.integers(0, 256, (H, W, 3)).astype(np.float64)
    for i in range(n):  # a slowly drifting pattern, so consecutive frames are related
        a = np.clip(np.roll(base, i, axis=1) + rng.normal(0, 8, (H, W, 3)), 0, 255).astype(np.uint8)
        Image.fromarray(a).save(os.path.join(d, "frame_%04d.png" % (i + 1)))


def test_evaluate_sintel_end_to_end(tmp_path):
    import gbvst
    from gbvst import sintel_eval as se
    from gbvst.options import default_opt
    from oracle import cpu_ref, prng
    gbvst._lib.load()
    H, W = 48, 64
    root = tmp_path / "sintel"
    _write_video(str(root / "training" / "final" / "alley_1"), 7, H, W, 1)
    _write_video(str(root / "test" / "final" / "ambush_1"), 6, H, W, 2)
    G = cpu_ref.RefResnetGenerator(3, 3, 8, 9)
    sd = prng.init_state_dict(cpu_ref.state_shapes(G), base_seed=2100)
    cpu_ref.load_np_state(G, sd)
    ck = tmp_path / "checkpoints" / "style1"
    os.makedirs(ck)
    for name in ("G_A", "G_B"):
        torch.save({k: torch.from_numpy(v) for k, v in sd.items()}, str(ck / ("latest_net_%s.pth" % name)))
    args = default_opt(False, ngf=8, checkpoints_dir=str(tmp_path / "checkpoints"), epoch="latest", gpu_ids=[0])
    out = tmp_path / "eval"
    st, lt, dt = se.evaluate_sintel(args, str(root), str(out), flow_model=_flow, num_domains=2)
    for name in ("TCL-ST", "TCL-LT", "DT"):
        assert (out / (name + ".json")).exists()
    # oracle on the same decoded frames
    for split, vid in (("training", "alley_1"), ("test", "ambush_1")):
        ds = se.SingleSintelVideo(str(root / split / "final" / vid))
        sts, lts = [], []
        with torch.no_grad():
            for i in range(len(ds)):
                img, last, past = (t.unsqueeze(0) if t.dim() == 3 else t for t in ds[i])
                x = G(img)
                png = np.asarray(Image.open(out / (vid + "_s1") / ("frame_%04d.png" % i))).astype(np.int32)
                want = (((x[0] + 1) / 2).clamp(0, 1) * 255 + 0.5).clamp(0, 255).permute(1, 2, 0).to(torch.uint8)
                assert np.abs(png - want.numpy().astype(np.int32)).max() <= 1
                for prev_img, vals in ((last, sts), (past, lts)):
                    if prev_img.dim() == 4:
                        ff, bf = _flow(prev_img, img), _flow(img, prev_img)
                        mask = cpu_ref.fbc_check(ff, bf)
                        vals.append(cpu_ref.tcl(x, G(prev_img), bf, mask).item())
        key = vid + "_s1"
        for got, ref in ((st["TCL-ST_" + key], np.mean(sts)), (lt["TCL-LT_" + key], np.mean(lts))):
            assert abs(got - ref) <= 1e-3 * abs(ref) + 1e-6, (key, got, ref)
    assert json.load(open(out / "TCL-ST.json"))["TCL-ST_mean"] == pytest.approx(np.mean(list(
        v for k, v in st.items() if not k.startswith("TCL-ST_mean"))), rel=1e-9)
