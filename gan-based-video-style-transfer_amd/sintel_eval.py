"""Temporal-consistency (TCL) evaluation, HIP-backed.

Drop-in for the metric path of methods/GAN-based/CycleGAN/sintel_eval.py:105-235 (and its
utils/sintel_eval.py:104-130 twin):
  computeTCL(net, flow_model, img_fake, img1, img2)
      = sqrt(mean((mask * (img_fake - warp(net.forward_eval(img2), bf)))^2)),
        ff = flow(img2 -> img1), bf = flow(img1 -> img2), mask = fbcCheckTorch(ff, bf)
  save_dict_as_json(out_id, data_dict, out_path, num_domains)
  SingleSintelVideo(vid_dir, transform, lt_len=5, crop_rows=None)
                        the per-video frame dataset (sintel_eval.py:63-103): sorted frame files,
                        items (img, img_last, img_past) with a 0-dim placeholder where a frame is
                        missing; crop_rows=432 is the utils/sintel_eval.py:82-88 variant
  sintel_transform      transforms.ToTensor() + Normalize(0.5, 0.5) restated (torchvision absent)
  save_image            vutils.save_image of denormalize(x) (sintel_eval.py:31-37) via PIL
  evaluate_video(...)   the per-video loop of evaluate_sintel (TCL-ST at i > 0, TCL-LT at i >= 5,
                        DT = generator time per frame in ms, synchronised), over any iterable of
                        (img, img_last, img_past) — a SingleSintelVideo or in-memory frames; writes
                        frame_%04d.png per frame when given a directory
  evaluate_sintel(...)  sintel_eval.py:143-235: every video of <sintel>/training/final and
                        test/final x styles 1..num_domains-1 (the checkpoints in sorted order), PNG
                        frames under <out>/<video>_s<y>/, then TCL-ST / TCL-LT / DT JSONs.

The flow estimator is a callable ``flow_model(a, b) -> [B, 2, H, W]``: the reference's
``computeRAFT(raft, a, b)`` is provided here on the HIP RAFT (``initRaftModel`` / ``computeRAFT``;
pretrained raft-chairs weights are not shipped, so they load only if a checkpoint is given), and any
other flow source plugs in the same way.  The TCL reduction itself is one fused kernel (vst_loss_temporal with lambda = 1:
warp + mask + squared error + fixed-order mean), the mask one vst_fbcheck launch.
"""
import json
import os
import time
from collections import OrderedDict

import numpy as np
import torch
import torch.utils.data

from . import ops


def tcl_from_flows(x_fake, prev_fake, ff, bf):
    """sqrt(mean((fbcheck(ff, bf) * (x_fake - warp(prev_fake, bf)))^2)) on NCHW 3-channel frames;
    returns a device scalar."""
    a = ops.nchw_to_nhwc(prev_fake.float().contiguous())
    b = ops.nchw_to_nhwc(x_fake.float().contiguous())
    bf = bf.float().contiguous()
    mask = ops.fbcheck(ff.float().contiguous(), bf)
    return torch.sqrt(ops.loss_temporal(a, b, bf, mask, 1.0, cl=x_fake.shape[1]))


def initRaftModel(opt=None, device="cuda", weights=None):
    """CycleGAN/sintel_eval.py:44-52: the full RAFT in eval mode.  ``weights``: a RAFT checkpoint
    (the reference loads raft/models/raft-chairs.pth, saved from nn.DataParallel — the "module."
    prefix is stripped), loaded with weights_only=True; without it the model keeps its random init
    (pretrained weights are not shipped with the reference)."""
    import argparse
    from .raft import RAFT
    args = opt if opt is not None else argparse.Namespace(small=False, mixed_precision=False, alternate_corr=False)
    model = RAFT(args)
    if weights is not None:
        sd = torch.load(weights, map_location="cpu", weights_only=True)
        model.load_state_dict({(k[7:] if k.startswith("module.") else k): v for k, v in sd.items()})
    return model.to(device).eval()


def computeRAFT(net, img1, img2, it=20, crop_rows=True):
    """CycleGAN/sintel_eval.py:54-60: InputPadder('sintel') + test-mode RAFT; returns flow_up cut to
    the first H rows (the reference's ``flow_up[:, :, :H, :]``, which keeps the top padding rows —
    SURVEY App. A; crop_rows=False returns the padded flow as utils/sintel_eval.py:62 does)."""
    from .raft import compute_raft
    H = img1.shape[2]
    flow_up = compute_raft(net, img1, img2, it=it)
    return flow_up[:, :, :H, :].contiguous() if crop_rows else flow_up


def computeTCL(net, flow_model, img_fake, img1, img2):
    """CycleGAN/sintel_eval.py:105-111 (net.forward_eval is the generator under test)."""
    ff_last = flow_model(img2, img1)
    bf_last = flow_model(img1, img2)
    with torch.no_grad():
        prev = net.forward_eval(img2)
    return tcl_from_flows(img_fake, prev, ff_last, bf_last)


def save_dict_as_json(out_id, data_dict, out_path, num_domains):
    """CycleGAN/sintel_eval.py:113-131: overall mean and per-style (_s<d>) means, then JSON."""
    dict_mean = 0
    dict_mean_s = np.zeros(num_domains - 1)
    for key, value in data_dict.items():
        len_3 = len(data_dict) / 3
        dict_mean += value / len(data_dict)
        for d in range(1, num_domains):
            if ("_s" + str(d)) in key:
                dict_mean_s[d - 1] += value / len_3
    data_dict[out_id + "_mean"] = float(dict_mean)
    for d in range(1, num_domains):
        data_dict[out_id + "_mean_s" + str(d)] = float(dict_mean_s[d - 1])
    os.makedirs(out_path, exist_ok=True)
    with open(os.path.join(out_path, out_id + ".json"), "w") as f:
        json.dump(data_dict, f, indent=4, sort_keys=False)
    return data_dict


def sintel_transform(pil_img):
    """transforms.ToTensor() + transforms.Normalize((0.5,)*3, (0.5,)*3) (sintel_eval.py:148-151):
    uint8 HWC -> float CHW / 255 -> (x - 0.5) / 0.5 (the same float ops torchvision runs)."""
    a = np.asarray(pil_img.convert("RGB"))
    t = torch.from_numpy(a.copy()).permute(2, 0, 1).contiguous().float().div(255)
    half = torch.tensor([0.5, 0.5, 0.5]).view(-1, 1, 1)
    return t.sub(half).div(half)


def denormalize(x):
    """sintel_eval.py:27-29."""
    return ((x + 1) / 2).clamp_(0, 1)


def save_image(x, ncol, filename):
    """sintel_eval.py:31-33: vutils.save_image(denormalize(x), nrow=ncol, padding=0) for one image:
    uint8(clamp(x * 255 + 0.5, 0, 255)) written as PNG."""
    from PIL import Image
    x = denormalize(x.detach().float().cpu().clone())
    nd = x.mul(255).add_(0.5).clamp_(0, 255).permute(1, 2, 0).to(torch.uint8).numpy()
    Image.fromarray(nd).save(filename)


class SingleSintelVideo(torch.utils.data.Dataset):
    """sintel_eval.py:63-103 (crop_rows=None: the CycleGAN copy, full 436 rows) /
    utils/sintel_eval.py:62-102 (crop_rows=432: frames cut to 432 rows, so RAFT needs no padding)."""

    def __init__(self, vid_dir, transform=sintel_transform, lt_len=5, crop_rows=None):
        self.vid_dir, self.transform, self.lt_len, self.crop_rows = vid_dir, transform, lt_len, crop_rows
        self.dataset = [os.path.join(vid_dir, f) for f in sorted(os.listdir(vid_dir))]
        self.num_images = len(self.dataset)

    def _load(self, fid):
        from PIL import Image
        img = self.transform(Image.open(fid))
        return img[:, :self.crop_rows, :] if self.crop_rows else img

    def __getitem__(self, index):
        img = self._load(self.dataset[index])
        last_img = torch.tensor(0, dtype=torch.long)
        past_img = torch.tensor(0, dtype=torch.long)
        if index > 0:
            last_img = self._load(self.dataset[index - 1])
        if index >= self.lt_len:
            past_img = self._load(self.dataset[index - self.lt_len])
        return img, last_img, past_img

    def __len__(self):
        return self.num_images


def evaluate_video(model, frames, flow_model, key, lt_len=5, tcl_st=None, tcl_lt=None, dt=None, vid_path=None,
                   device="cuda"):
    """One video of evaluate_sintel (sintel_eval.py:196-229).  frames: a SingleSintelVideo (items
    (img, img_last, img_past)) or a list of [1,3,H,W] / [3,H,W] images in [-1, 1]; fills the
    OrderedDicts TCL-ST_<key>, TCL-LT_<key>, DT_<key> with the per-video means and, given vid_path,
    writes frame_%04d.png per stylised frame.  DT is device-synchronised (the reference's is not)."""
    tcl_st = OrderedDict() if tcl_st is None else tcl_st
    tcl_lt = OrderedDict() if tcl_lt is None else tcl_lt
    dt = OrderedDict() if dt is None else dt
    if vid_path is not None:
        os.makedirs(vid_path, exist_ok=True)
    batched = lambda t: (t if t.dim() == 4 else t.unsqueeze(0)).to(device)  # noqa: E731
    st_vals, lt_vals, dt_vals = [], [], []
    for i in range(len(frames)):
        item = frames[i]
        if isinstance(item, (tuple, list)):
            img, img_last, img_past = (batched(t) if t.dim() >= 3 else None for t in item)
        else:
            img = batched(item)
            img_last = batched(frames[i - 1]) if i > 0 else None
            img_past = batched(frames[i - lt_len]) if i >= lt_len else None
        torch.cuda.synchronize()
        t0 = time.time()
        x_fake = model.forward_eval(img)
        torch.cuda.synchronize()
        dt_vals.append((time.time() - t0) * 1000)
        if i > 0:
            st_vals.append(float(computeTCL(model, flow_model, x_fake, img, img_last)))
        if i >= lt_len:
            lt_vals.append(float(computeTCL(model, flow_model, x_fake, img, img_past)))
        if vid_path is not None:
            save_image(x_fake[0], 1, os.path.join(vid_path, "frame_%04d.png" % i))
    tcl_st["TCL-ST_" + key] = float(np.array(st_vals).mean()) if st_vals else float("nan")
    tcl_lt["TCL-LT_" + key] = float(np.array(lt_vals).mean()) if lt_vals else float("nan")
    dt["DT_" + key] = float(np.array(dt_vals).mean())
    return tcl_st, tcl_lt, dt


def evaluate_sintel(args, sintel_dir, out_path, flow_model=None, num_domains=4, crop_rows=None, lt_len=5,
                    raft_weights=None, device="cuda"):
    """sintel_eval.py:143-235: for every video of <sintel_dir>/training/final then test/final and
    every style y = 1..num_domains-1, load the y-th checkpoint directory of args.checkpoints_dir
    (sorted; create_model + setup, which loads '<epoch>_net_G_A.pth'), run forward_eval frame by
    frame (PNG per frame under out_path/<video>_s<y>/), TCL-ST / TCL-LT through flow_model (default:
    the HIP RAFT, initRaftModel / computeRAFT, 20 iterations) and fb-check, then write TCL-ST.json,
    TCL-LT.json and DT.json with save_dict_as_json.  Returns the three dicts."""
    from .models import create_model
    if flow_model is None:
        raft = initRaftModel(device=device, weights=raft_weights)
        flow_model = lambda a, b: computeRAFT(raft, a, b, crop_rows=crop_rows is None)  # noqa: E731
    videos = []
    for split in ("training", "test"):
        d = os.path.join(sintel_dir, split, "final")
        if os.path.isdir(d):
            videos += [(v, os.path.join(d, v)) for v in sorted(os.listdir(d))]
    model_list = sorted(os.listdir(args.checkpoints_dir))
    tcl_st, tcl_lt, dt = OrderedDict(), OrderedDict(), OrderedDict()
    for vid, vid_dir in videos:
        dset = SingleSintelVideo(vid_dir, sintel_transform, lt_len, crop_rows)
        for y in range(1, num_domains):
            key = vid + "_s" + str(y)
            args.name = model_list[y - 1]
            model = create_model(args)
            model.setup(args)
            evaluate_video(model, dset, flow_model, key, lt_len, tcl_st, tcl_lt, dt,
                           vid_path=os.path.join(out_path, key), device=device)
    save_dict_as_json("TCL-ST", tcl_st, out_path, num_domains)
    save_dict_as_json("TCL-LT", tcl_lt, out_path, num_domains)
    save_dict_as_json("DT", dt, out_path, num_domains)
    return tcl_st, tcl_lt, dt
