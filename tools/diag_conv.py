"""Diagnostic: fwd / dgrad / wgrad error vs fp64 per conv arithmetic on the VGG16 layer shapes."""
import sys, os
R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, R)
import torch, torch.nn.functional as F
import gbvst
from gbvst import ops
gbvst._lib.load()
B = int(os.environ.get("B", "2")); S = int(os.environ.get("S", "32"))
shapes = [(3, 64, S), (64, 64, S), (64, 128, S // 2), (128, 128, S // 2), (128, 256, S // 4), (256, 256, S // 4),
          (256, 512, S // 8), (512, 512, S // 8)]
g = torch.Generator().manual_seed(0)
for ci, co, hw in shapes:
    x = torch.randn(B, ci, hw, hw, generator=g, dtype=torch.float64)
    w = torch.randn(co, ci, 3, 3, generator=g, dtype=torch.float64) * (2.0 / (9 * ci)) ** 0.5
    gy = torch.randn(B, co, hw, hw, generator=g, dtype=torch.float64)
    y64 = F.conv2d(x, w, padding=1)
    dx64 = F.conv_transpose2d(gy, w, padding=1)
    xn = ops.nchw_to_nhwc(x.float().cuda()); gyn = ops.nchw_to_nhwc(gy.float().cuda())
    kc = ops.weight_pack(w.float().cuda(), ops.PACK_FWD); ck = ops.weight_pack(w.float().cuda(), ops.PACK_DGRAD)
    row = []
    for pol in ("fp32", "bf16x3", "bf16x6"):
        ops.set_conv_math(pol)
        y = ops.nhwc_to_nchw(ops.conv2d_fwd(xn, kc, None, ops.cpad(co), 3, 3, 1, 1, "zero", role="fwd"), co).double().cpu()
        dx = ops.nhwc_to_nchw(ops.conv2d_tfwd(gyn, ck, None, hw, hw, ops.cpad(ci), 3, 3, 1, 1, role="fwd"), ci).double().cpu()
        e = lambda a, b: float((a - b).abs().max() / b.abs().max())
        row.append("%s fwd %.1e dgrad %.1e" % (pol, e(y, y64), e(dx, dx64)))
    print(ci, co, hw, " | ".join(row), flush=True)
