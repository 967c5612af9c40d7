"""train.py end to end on the GPU (SURVEY §5 loss log, train.py:57-130): two epochs of the HIP CycleGAN
step on synthetic FC2 batches — the loss log gets the reference's line format with finite losses, the
checkpoints land under the reference's names and load back (weights_only) into a fresh model."""
import math
import os
import re

import pytest
import torch

pytestmark = pytest.mark.gpu


def test_train_main_synthetic(tmp_path):
    import gbvst.train as T
    argv = ["--synthetic", "4", "--batch_size", "2", "--crop_size", "64", "--ngf", "8", "--ndf", "8",
            "--n_epochs", "1", "--n_epochs_decay", "1", "--print_freq", "2", "--save_latest_freq", "4",
            "--save_epoch_freq", "1", "--pool_size", "0", "--checkpoints_dir", str(tmp_path), "--name", "t"]
    assert T.main(argv) == 0
    d = os.path.join(str(tmp_path), "t")
    lines = open(os.path.join(d, "loss_log.txt")).read().splitlines()[1:]
    assert len(lines) == 4  # 2 epochs x 4 images / print_freq 2
    pat = re.compile(r"^\(epoch: (\d+), iters: (\d+), time: [0-9.]+, data: [0-9.]+\) ((\w+: -?[0-9.]+ )+)$")
    for ln in lines:
        m = pat.match(ln)
        assert m, ln
        vals = [float(v) for v in re.findall(r": (-?[0-9.]+)", m.group(3))]
        assert all(math.isfinite(v) for v in vals)
    for f in ("latest_net_G_A.pth", "1_net_D_B.pth", "2_net_G_B.pth"):
        assert os.path.exists(os.path.join(d, f)), f
    sd = torch.load(os.path.join(d, "2_net_G_A.pth"), map_location="cpu", weights_only=True)
    assert all(torch.isfinite(v).all() for v in sd.values())
