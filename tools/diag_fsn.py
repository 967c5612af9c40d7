"""Developer diagnostic: the FastStyleNet data-gradient ops (conv2d_tfwd on the golden test's shapes)
under bf16x6 vs the fp32 policy — norm-wise relative difference per op."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import gbvst  # noqa: E402
from gbvst import ops  # noqa: E402

gbvst._lib.load()
dev = torch.device("cuda")
g = torch.Generator().manual_seed(0)


def rel(a, b):
    return float((a - b).norm() / b.norm())


cases = [  # name, N, Hin, Win, Cin(x), Cout(dy), k, st
    ("deconv3", 2, 32, 40, 32, 3, 9, 1), ("deconv2", 2, 32, 40, 64, 32, 3, 1),
    ("deconv1", 2, 16, 20, 128, 64, 3, 1), ("res", 2, 8, 10, 128, 128, 3, 1),
    ("conv3", 2, 16, 20, 64, 128, 3, 2), ("conv2", 2, 32, 40, 32, 64, 3, 2), ("conv1", 2, 32, 40, 3, 32, 9, 1)]
for name, N, H, W, Ci, Co, k, st in cases:
    w = (torch.randn(Co, Ci, k, k, generator=g) * 0.05).to(dev)
    ck = ops.weight_pack(w, ops.PACK_DGRAD)
    Ho, Wo = (H + st - 1) // st, (W + st - 1) // st
    dy = torch.randn(N, Ho, Wo, ops.cpad(Co), generator=g).to(dev)
    dy[..., Co:] = 0
    p = k // 2
    res = {}
    for m in ("fp32", "bf16x6", "bf16x3"):
        ops.set_conv_math(m)
        if st == 1:
            dx = ops.conv2d_tfwd(dy, ck, None, H, W, ops.cpad(Ci), k, k, 1, p, pad_mode="reflect")
        else:
            dxp = ops.conv2d_tfwd(dy, ck, None, H + 2 * p, W + 2 * p, ops.cpad(Ci), k, k, st, 0)
            dx = ops.reflect_fold(dxp, p, None)
        res[m] = dx.clone()
    print(name, "x6 vs fp32 %.2e" % rel(res["bf16x6"], res["fp32"]), "x3 vs fp32 %.2e" % rel(res["bf16x3"], res["fp32"]),
          flush=True)
