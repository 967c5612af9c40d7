"""Temporal-consistency (TCL) evaluation, HIP-backed.

Drop-in for the metric path of methods/GAN-based/CycleGAN/sintel_eval.py:105-235 (and its
utils/sintel_eval.py:104-130 twin):
  computeTCL(net, flow_model, img_fake, img1, img2)
      = sqrt(mean((mask * (img_fake - warp(net.forward_eval(img2), bf)))^2)),
        ff = flow(img2 -> img1), bf = flow(img1 -> img2), mask = fbcCheckTorch(ff, bf)
  save_dict_as_json(out_id, data_dict, out_path, num_domains)
  evaluate_video(...)   the per-video loop of evaluate_sintel (TCL-ST at i > 0, TCL-LT at i >= 5,
                        DT = generator time per frame in ms), over in-memory frames.

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


def evaluate_video(model, frames, flow_model, key, lt_len=5, tcl_st=None, tcl_lt=None, dt=None):
    """One video of evaluate_sintel (sintel_eval.py:203-229): frames is a list of [1,3,H,W] images
    in [-1, 1]; fills OrderedDicts TCL-ST_<key>, TCL-LT_<key>, DT_<key> with the per-video means."""
    tcl_st = OrderedDict() if tcl_st is None else tcl_st
    tcl_lt = OrderedDict() if tcl_lt is None else tcl_lt
    dt = OrderedDict() if dt is None else dt
    st_vals, lt_vals, dt_vals = [], [], []
    for i, img in enumerate(frames):
        torch.cuda.synchronize()
        t0 = time.time()
        x_fake = model.forward_eval(img)
        torch.cuda.synchronize()
        dt_vals.append((time.time() - t0) * 1000)
        if i > 0:
            st_vals.append(float(computeTCL(model, flow_model, x_fake, img, frames[i - 1])))
        if i >= lt_len:
            lt_vals.append(float(computeTCL(model, flow_model, x_fake, img, frames[i - lt_len])))
    tcl_st["TCL-ST_" + key] = float(np.array(st_vals).mean()) if st_vals else float("nan")
    tcl_lt["TCL-LT_" + key] = float(np.array(lt_vals).mean()) if lt_vals else float("nan")
    dt["DT_" + key] = float(np.array(dt_vals).mean())
    return tcl_st, tcl_lt, dt
