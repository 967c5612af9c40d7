"""Pin the StarGAN oracle (oracle/stargan_ref.py) against fixtures the reference itself produced
(oracle/gen_golden_stargan.py imported methods/GAN-based/StarGAN/model.py).  CPU only."""
import numpy as np
import torch

from oracle import prng, stargan_ref

CFG = dict(image_size=32, c_dim=4, conv_dim=8, g_repeat=2, d_repeat=4)


def _rel(got, ref):
    got, ref = np.asarray(got, np.float64), np.asarray(ref, np.float64)
    return np.abs(got - ref).max() / (np.abs(ref).max() + 1e-30)


def make_ref(which):
    c = CFG
    if which == "G":
        net = stargan_ref.RefGenerator(c["conv_dim"], c["c_dim"], c["g_repeat"])
        base = 700
    else:
        net = stargan_ref.RefDiscriminator(c["image_size"], c["conv_dim"], c["c_dim"], c["d_repeat"])
        base = 710
    net.load_state_dict({k: torch.from_numpy(np.asarray(v)) for k, v in stargan_ref.sg_weights(net, base).items()})
    return net


def test_generator_matches_reference(golden):
    g = golden("stargan_small")
    G = make_ref("G").train()
    x = torch.from_numpy(g["x"]).requires_grad_(True)
    c = stargan_ref.label2onehot(torch.from_numpy(g["lab"]), CFG["c_dim"])
    y = G(x, c)
    assert _rel(y.detach().numpy(), g["g_y"]) < 1e-5
    (y * torch.from_numpy(prng.normal(702, tuple(y.shape)))).sum().backward()
    assert _rel(x.grad.numpy(), g["g_dx"]) < 1e-4
    for k, p in G.named_parameters():
        assert _rel(p.grad.numpy(), g["g_g_" + k]) < 1e-4, k
    for k, b in G.named_buffers():
        np.testing.assert_allclose(b.numpy(), g["g_rb_" + k], rtol=1e-5, atol=1e-6)
    Ge = make_ref("G").eval()
    with torch.no_grad():
        assert _rel(Ge(torch.from_numpy(g["x"]), c).numpy(), g["g_y_eval"]) < 1e-5


def test_discriminator_and_penalty_match_reference(golden):
    g = golden("stargan_small")
    D = make_ref("D")
    x = torch.from_numpy(g["d_x"]).requires_grad_(True)
    src, cls = D(x)
    assert _rel(src.detach().numpy(), g["d_src"]) < 1e-5
    assert _rel(cls.detach().numpy(), g["d_cls"]) < 1e-5
    ((src * torch.from_numpy(prng.normal(712, tuple(src.shape)))).sum()
     + (cls * torch.from_numpy(prng.normal(713, tuple(cls.shape)))).sum()).backward()
    assert _rel(x.grad.numpy(), g["d_dx"]) < 1e-5
    for k, p in D.named_parameters():
        assert _rel(p.grad.numpy(), g["d_g_" + k]) < 1e-5, k
    D = make_ref("D")
    xh = torch.from_numpy(g["d_x"]).requires_grad_(True)
    src, _ = D(xh)
    gp = stargan_ref.gradient_penalty(src, xh)
    gp.backward()
    np.testing.assert_allclose(gp.item(), float(g["gp"]), rtol=1e-5)
    for k, p in D.named_parameters():
        if "gp_g_" + k in g.files:
            assert _rel(p.grad.numpy(), g["gp_g_" + k]) < 1e-4, k
        else:
            assert p.grad is None, k


def test_train_iterations_match_reference(golden):
    g = golden("stargan_small")
    G, D = make_ref("G").train(), make_ref("D").train()
    g_opt = torch.optim.Adam(G.parameters(), 1e-4, [0.5, 0.999])
    d_opt = torch.optim.Adam(D.parameters(), 1e-4, [0.5, 0.999])
    for i in range(3):
        alpha = torch.from_numpy(prng.uniform_f32(730 + i, (2, 1, 1, 1)))
        ls = stargan_ref.train_iteration(G, D, g_opt, d_opt, torch.from_numpy(g["t_x"]),
                                         torch.from_numpy(g["t_lorg"]), torch.from_numpy(g["t_ltrg"]), alpha, i,
                                         CFG["c_dim"], n_critic=2)
        got = np.array([ls.get(k, np.nan) for k in stargan_ref.LOSS_KEYS])
        np.testing.assert_allclose(got, g["t_losses"][i], rtol=1e-4, atol=1e-6)
