"""Diagnostic: Johnson step-0 gradient error per conv arithmetic policy (GPU)."""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
import numpy as np, torch
import gbvst
from gbvst import ops, faststyle, perceptual
from oracle import prng
import test_gpu_style as T
g = np.load("tests/golden/style_small.npz")
emph = tuple(float(v) for v in g["js_emph"])
for pol in ("fp32", "bf16x6", "bf16x3", "mixed"):
    ops.set_conv_math(pol)
    model = T._fsn(gbvst, 540)
    vgg = T._vgg(gbvst, "vgg16", 550)
    J = faststyle.Johnson([torch.from_numpy(g["js_style"])], emphasis=emph, lr=1e-3, batch_sz=2, device="cuda", vgg=vgg, model=model)
    x = ops.nchw_to_nhwc(torch.from_numpy(g["js_img"]).cuda())
    J.adam.zero_grad()
    loss, cl, sl, tv, styled = J.losses_nhwc(x)
    loss.backward()
    params = dict(model.named_parameters())
    errs = {k[5:]: T._rel(params[k[5:]].grad, g[k]) for k in g.files if k.startswith("js_g_")}
    print(pol, "losses", [float(v) for v in (loss, cl, sl, tv)], "ref", list(g["js_losses"][0]))
    print(pol, {k: "%.2e" % v for k, v in errs.items()})
    # style-only / content-only decomposition of the conv1 gradient error
    for name, which in (("content", 1), ("style", 2), ("tv", 3)):
        J.adam.zero_grad()
        out = J.losses_nhwc(x)
        out[which].backward()
        print(pol, name, "conv1 grad norm", float(params["conv1.conv2d.weight"].grad.norm()))
