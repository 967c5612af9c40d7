"""Developer diagnostic: after an in-place weight update, every pack refreshed by ops.PackBatch must
equal a fresh single pack of the current weight (FastStyleNet, ResnetGenerator, PatchGAN D)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import gbvst  # noqa: E402
from gbvst import faststyle, networks, ops  # noqa: E402

gbvst._lib.load()
dev = torch.device("cuda")


def walk(P, path=""):
    if isinstance(P, dict):
        for k, v in P.items():
            yield from walk(v, path + "/" + str(k))
    elif isinstance(P, (list, tuple)):
        for i, v in enumerate(P):
            yield from walk(v, path + "[%d]" % i)
    elif torch.is_tensor(P):
        yield path, P


for name, net in (("fsn", faststyle.FastStyleNet(3, 1).to(dev)),
                  ("G", networks.define_G(3, 3, 16, "resnet_9blocks", "instance", False, "normal", 0.02, [0])),
                  ("D", networks.define_D(3, 16, "basic", 3, "instance", "normal", 0.02, [0]))):
    P = net.packs()
    before = {k: (t.clone(), t.vst_split.clone() if hasattr(t, "vst_split") else None) for k, t in walk(P)}
    with torch.no_grad():
        net.flat_param.mul_(1.5).add_(0.01)
    net.bump_version()
    P2 = net.packs()
    assert P2 is P
    os.environ["VST_PACK_BATCH"] = "0"
    networks.PACK_BATCH = False
    saved = net._packs
    net._packs = None
    Q = net.packs()
    networks.PACK_BATCH = True
    net._packs = saved
    fresh = dict(walk(Q))
    bad = 0
    for k, t in walk(P2):
        f = fresh[k]
        d = float((t - f).abs().max())
        ds = float((t.vst_split.float() - f.vst_split.float()).abs().max()) if hasattr(t, "vst_split") else 0.0
        chg = float((t - before[k][0]).abs().max())
        if d > 0 or ds > 0:
            bad += 1
            print(name, k, tuple(t.shape), "diff %.3e split %.3e changed %.3e" % (d, ds, chg))
    print(name, "packs", len(fresh), "mismatching", bad, flush=True)
