"""Diagnostic: where do the fp32 and bf16x6 conv policies diverge in the Johnson step? (GPU)"""
import sys, os
R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, R); sys.path.insert(0, os.path.join(R, "tests"))
import numpy as np, torch
import gbvst
from gbvst import ops, faststyle, perceptual
import test_gpu_style as T
g = np.load("tests/golden/style_small.npz")
emph = tuple(float(v) for v in g["js_emph"])
res = {}
for pol in ("fp32", "bf16x6"):
    ops.set_conv_math(pol)
    model = T._fsn(gbvst, 540)
    vgg = T._vgg(gbvst, "vgg16", 550)
    J = faststyle.Johnson([torch.from_numpy(g["js_style"])], emphasis=emph, lr=1e-3, batch_sz=2, device="cuda", vgg=vgg, model=model)
    x = ops.nchw_to_nhwc(torch.from_numpy(g["js_img"]).cuda())
    d = {}
    d["style_gram"] = [t.clone() for t in J.styles[0]]
    _, styled = model.forward_nhwc(x)
    d["styled"] = styled.detach().clone()
    s_in = perceptual.normalize_nhwc(styled.detach(), d0=255.0).requires_grad_(True)
    feats = vgg.forward_nhwc(s_in)
    d["feats"] = [f.detach().clone() for f in feats]
    grams = [perceptual.gram_nhwc(f) for f in feats]
    d["grams"] = [t.detach().clone() for t in grams]
    sl = sum(perceptual.mse_loss(G, gs, emph[1]) for G, gs in zip(grams, J._style_targets(2)))
    sl.backward()
    d["dstyled_in"] = s_in.grad.clone()
    # per-level gradient wrt each VGG feature
    feats2 = vgg.forward_nhwc(s_in.detach())
    fs = [f.detach().requires_grad_(True) for f in feats2]
    sl2 = sum(perceptual.mse_loss(perceptual.gram_nhwc(f), gs, emph[1]) for f, gs in zip(fs, J._style_targets(2)))
    sl2.backward()
    d["dfeat"] = [f.grad.clone() for f in fs]
    res[pol] = d
def rel(a, b):
    return float((a - b).abs().max() / (b.abs().max() + 1e-30))
A, B = res["bf16x6"], res["fp32"]
print("styled", rel(A["styled"], B["styled"]))
for i in range(4):
    print("level", i, "style_gram", rel(A["style_gram"][i], B["style_gram"][i]), "feat", rel(A["feats"][i], B["feats"][i]),
          "gram", rel(A["grams"][i], B["grams"][i]), "dfeat", rel(A["dfeat"][i], B["dfeat"][i]),
          "G-Gs rel", float((B["grams"][i][0]-B["style_gram"][i][0]).abs().max()/B["grams"][i].abs().max()))
print("dstyled_in", rel(A["dstyled_in"], B["dstyled_in"]))
