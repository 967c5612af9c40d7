"""Pin the style/RAFT oracle (oracle/style_ref.py) against fixtures the reference itself produced
(oracle/gen_golden_style.py imported methods/learning-based/{fs_lib,network}.py and
utils/raft/raft/corr.py).  CPU only."""
import numpy as np
import torch

from oracle import prng, style_ref


def _rel(got, ref):
    got, ref = np.asarray(got, np.float64), np.asarray(ref, np.float64)
    return np.abs(got - ref).max() / (np.abs(ref).max() + 1e-30)


def test_fs_warp_matches_reference(golden):
    g = golden("style_small")
    for case in ("zero", "frac", "oob"):
        x = torch.from_numpy(g["fsw_x"]).requires_grad_(True)
        y = style_ref.fs_warp(x, torch.from_numpy(g[f"fsw_{case}_flow"]))
        y.backward(torch.from_numpy(g["fsw_gout"]))
        np.testing.assert_allclose(y.detach().numpy(), g[f"fsw_{case}_y"], rtol=0, atol=1e-6)
        np.testing.assert_allclose(x.grad.numpy(), g[f"fsw_{case}_dx"], rtol=0, atol=1e-6)
    # the far out-of-range case really exercises the validity mask
    assert (g["fsw_oob_y"] == 0).mean() > 0.3


def test_vgg_matches_reference(golden):
    g = golden("style_small")
    for arch, base in (("vgg16", 510), ("vgg19", 520)):
        net = style_ref.RefVGG(arch)
        style_ref.load_np(net, style_ref.vgg_weights(net, base))
        x = torch.from_numpy(g[f"{arch}_x"]).requires_grad_(True)
        ys = net(x)
        loss = 0
        for i, y in enumerate(ys):
            assert _rel(y.detach().numpy(), g[f"{arch}_y{i}"]) < 1e-5, (arch, i)
            loss = loss + (y * torch.from_numpy(prng.normal(base + 10 + i, tuple(y.shape)))).sum()
        loss.backward()
        assert _rel(x.grad.numpy(), g[f"{arch}_dx"]) < 1e-5, arch


def test_faststylenet_matches_reference(golden):
    g = golden("style_small")
    net = style_ref.RefFastStyleNet(3)
    style_ref.load_np(net, style_ref.fsn_weights(net, 530))
    x = torch.from_numpy(g["fsn_x"]).requires_grad_(True)
    feats, img = net(x, 0.8)
    assert _rel(feats.detach().numpy(), g["fsn_feats"]) < 1e-5
    assert _rel(img.detach().numpy(), g["fsn_img"]) < 1e-5
    gf = torch.from_numpy(prng.normal(532, tuple(feats.shape)))
    gi = torch.from_numpy(prng.normal(533, tuple(img.shape)))
    ((feats * gf).sum() + (img * gi).sum()).backward()
    assert _rel(x.grad.numpy(), g["fsn_dx"]) < 1e-4
    names = [k[len("fsn_g_"):] for k in g.files if k.startswith("fsn_g_")]
    assert len(names) > 40
    params = dict(net.named_parameters())
    for k in names:
        assert _rel(params[k].grad.numpy(), g["fsn_g_" + k]) < 1e-3, k


def test_johnson_step_matches_reference(golden):
    g = golden("style_small")
    model = style_ref.RefFastStyleNet(3)
    style_ref.load_np(model, style_ref.fsn_weights(model, 540))
    vgg = style_ref.RefVGG("vgg16")
    style_ref.load_np(vgg, style_ref.vgg_weights(vgg, 550))
    with torch.no_grad():
        grams = [style_ref.gram_matrix(f) for f in vgg(style_ref.normalize(torch.from_numpy(g["js_style"])))]
    adam = torch.optim.Adam(model.parameters(), lr=1e-3)
    emph = tuple(float(v) for v in g["js_emph"])
    params = dict(model.named_parameters())
    for s in range(2):
        adam.zero_grad()
        ls = style_ref.johnson_losses(model, vgg, torch.from_numpy(g["js_img"]), grams, *emph)
        ls[0].backward()
        np.testing.assert_allclose([float(v) for v in ls], g["js_losses"][s], rtol=1e-4)
        if s == 0:
            for k in [k[len("js_g_"):] for k in g.files if k.startswith("js_g_")]:
                assert _rel(params[k].grad.numpy(), g["js_g_" + k]) < 1e-3, k
        adam.step()


def test_corr_block_matches_reference(golden):
    g = golden("corr_small")
    cb = style_ref.RefCorrBlock(torch.from_numpy(g["f1"]), torch.from_numpy(g["f2"]), 4, 4)
    for i in range(4):
        np.testing.assert_allclose(cb.pyr[i].numpy(), g[f"level{i}"], rtol=1e-5, atol=1e-5)
    out = cb(torch.from_numpy(g["coords"]))
    np.testing.assert_allclose(out.numpy(), g["lookup"], rtol=1e-5, atol=1e-5)
    # some window samples fall outside the map (zeros padding is exercised)
    assert (g["lookup"] == 0).mean() > 0.01
