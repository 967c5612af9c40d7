"""CPU oracle for RAFT inference (SURVEY §8 A19 + §8f rank 3).

TEST INFRASTRUCTURE ONLY (see oracle/__init__.py): a functional stock-PyTorch CPU restatement of
the full RAFT model evaluated from a state_dict, pinned against tests/golden/raft_small.npz, which
oracle/gen_golden_raft.py wrote by importing the reference utils/raft/raft/raft.py.

Reference files restated (paths relative to the reference root):
  utils/raft/raft/extractor.py:6-53, 117-189   ResidualBlock, BasicEncoder (instance / batch norm)
  utils/raft/raft/update.py:6-13, 32-58, 82-139 FlowHead, SepConvGRU, BasicMotionEncoder,
                                                BasicUpdateBlock (mask head * 0.25)
  utils/raft/raft/raft.py:63-144               initialize_flow, upsample_flow, forward
  utils/raft/raft/utils/utils.py:7-24           InputPadder (replicate)
  utils/raft/raft/corr.py                      via oracle/style_ref.RefCorrBlock (already pinned)
"""
import numpy as np
import torch
import torch.nn.functional as F

from oracle.style_ref import RefCorrBlock


def _conv(sd, name, x, stride=1, padding=0):
    return F.conv2d(x, sd[name + ".weight"], sd.get(name + ".bias"), stride=stride, padding=padding)


def _norm(sd, name, x, kind):
    if kind == "instance":
        return F.instance_norm(x, eps=1e-5)
    if kind == "batch":
        return F.batch_norm(x, sd[name + ".running_mean"], sd[name + ".running_var"], sd[name + ".weight"],
                            sd[name + ".bias"], False, 0.0, 1e-5)
    return x


def encoder(sd, pre, x, kind):
    """BasicEncoder.forward (eval)."""
    y = F.relu(_norm(sd, pre + "norm1", _conv(sd, pre + "conv1", x, 2, 3), kind))
    for li, stride in ((1, 1), (2, 2), (3, 2)):
        for bi in range(2):
            b = "%slayer%d.%d." % (pre, li, bi)
            s = stride if bi == 0 else 1
            t = F.relu(_norm(sd, b + "norm1", _conv(sd, b + "conv1", y, s, 1), kind))
            t = F.relu(_norm(sd, b + "norm2", _conv(sd, b + "conv2", t, 1, 1), kind))
            if b + "downsample.0.weight" in sd:
                y = _norm(sd, b + "norm3", _conv(sd, b + "downsample.0", y, s, 0), kind)
            y = F.relu(y + t)
    return _conv(sd, pre + "conv2", y)


def update_block(sd, net, inp, corr, flow, want_mask=True):
    u = "update_block."
    cor = F.relu(_conv(sd, u + "encoder.convc1", corr))
    cor = F.relu(_conv(sd, u + "encoder.convc2", cor, 1, 1))
    flo = F.relu(_conv(sd, u + "encoder.convf1", flow, 1, 3))
    flo = F.relu(_conv(sd, u + "encoder.convf2", flo, 1, 1))
    out = F.relu(_conv(sd, u + "encoder.conv", torch.cat([cor, flo], 1), 1, 1))
    x = torch.cat([inp, out, flow], 1)
    h = net
    for sfx, pad in (("1", (0, 2)), ("2", (2, 0))):
        hx = torch.cat([h, x], 1)
        z = torch.sigmoid(_conv(sd, u + "gru.convz" + sfx, hx, 1, pad))
        r = torch.sigmoid(_conv(sd, u + "gru.convr" + sfx, hx, 1, pad))
        q = torch.tanh(_conv(sd, u + "gru.convq" + sfx, torch.cat([r * h, x], 1), 1, pad))
        h = (1 - z) * h + z * q
    delta = _conv(sd, u + "flow_head.conv2", F.relu(_conv(sd, u + "flow_head.conv1", h, 1, 1)), 1, 1)
    mask = None
    if want_mask:
        mask = 0.25 * _conv(sd, u + "mask.2", F.relu(_conv(sd, u + "mask.0", h, 1, 1)))
    return h, mask, delta


def coords_grid(b, h, w, dtype=torch.float32):
    ys, xs = torch.meshgrid(torch.arange(h), torch.arange(w), indexing="ij")
    return torch.stack([xs, ys], 0).to(dtype)[None].repeat(b, 1, 1, 1)


def upsample_flow(flow, mask):
    n, _, h, w = flow.shape
    m = torch.softmax(mask.view(n, 1, 9, 8, 8, h, w), dim=2)
    up = F.unfold(8 * flow, [3, 3], padding=1).view(n, 2, 9, 1, 1, h, w)
    up = torch.sum(m * up, dim=2).permute(0, 1, 4, 2, 5, 3)
    return up.reshape(n, 2, 8 * h, 8 * w)


def pad_replicate(x, pads):
    return F.pad(x, list(pads), mode="replicate")


def input_pads(shape, mode="sintel"):
    ht, wd = shape[-2:]
    pad_ht = (((ht // 8) + 1) * 8 - ht) % 8
    pad_wd = (((wd // 8) + 1) * 8 - wd) % 8
    if mode == "sintel":
        return (pad_wd // 2, pad_wd - pad_wd // 2, pad_ht // 2, pad_ht - pad_ht // 2)
    return (pad_wd // 2, pad_wd - pad_wd // 2, 0, pad_ht)


def raft_forward(sd, image1, image2, iters=12, flow_init=None, test_mode=False, with_features=False):
    """raft.py:86-144 (full model, fp32, eval)."""
    image1 = 2 * (image1 / 255.0) - 1.0
    image2 = 2 * (image2 / 255.0) - 1.0
    b = image1.shape[0]
    fm = encoder(sd, "fnet.", torch.cat([image1, image2], 0), "instance")
    fmap1, fmap2 = fm[:b], fm[b:]
    corr_fn = RefCorrBlock(fmap1, fmap2, 4, 4)
    c = encoder(sd, "cnet.", image1, "batch")
    net, inp = torch.tanh(c[:, :128]), torch.relu(c[:, 128:])
    h8, w8 = c.shape[-2:]
    coords0, coords1 = coords_grid(b, h8, w8, fmap1.dtype), coords_grid(b, h8, w8, fmap1.dtype)
    if flow_init is not None:
        coords1 = coords1 + flow_init
    preds = []
    for it in range(iters):
        corr = corr_fn(coords1)
        flow = coords1 - coords0
        net, mask, delta = update_block(sd, net, inp, corr, flow, want_mask=(not test_mode or it == iters - 1))
        coords1 = coords1 + delta
        if mask is not None:
            preds.append(upsample_flow(coords1 - coords0, mask))
    feats = (fmap1, fmap2, c) if with_features else None
    if test_mode:
        out = (coords1 - coords0, preds[-1])
    else:
        out = preds
    return (out, feats) if with_features else out


# ------------------------------------------------------------------- fixture weights (PRNG)
def raft_weights(state_shapes, base, flow_scale=1.0):
    """Counter-PRNG state_dict by name: conv weights N(0, 1/fan_in), conv biases N(0, 0.05), BN
    gamma N(1, 0.1), beta N(0, 0.1), running_mean N(0, 0.1), running_var U(0.5, 1.5).  flow_scale
    multiplies the flow head's last conv (small, smooth flows keep fbcCheck masks non-trivial)."""
    from oracle import prng
    sd = {}
    for k, shape in state_shapes.items():
        # downsample.1 is the same BatchNorm module as norm3 (extractor.py:46-51): one value for both
        s = prng.seed_for(k.replace("downsample.1.", "norm3."), base)
        shape = tuple(shape)
        if k.endswith("num_batches_tracked"):
            sd[k] = np.array(0, dtype=np.int64)
        elif k.endswith("running_mean"):
            sd[k] = prng.normal(s, shape, std=0.1)
        elif k.endswith("running_var"):
            sd[k] = prng.uniform_f32(s, shape, 0.5, 1.5)
        elif len(shape) == 4:
            sd[k] = prng.normal(s, shape, std=(1.0 / np.prod(shape[1:])) ** 0.5)
        elif "norm" in k or "downsample.1" in k:
            sd[k] = prng.normal(s, shape, std=0.1, mean=1.0 if k.endswith("weight") else 0.0)
        else:
            sd[k] = prng.normal(s, shape, std=0.05)
        if k.startswith("update_block.flow_head.conv2."):
            sd[k] = (sd[k] * np.float32(flow_scale)).astype(np.float32)
    return sd
