"""Pin the C3 oracle (oracle/c3_ref.py: CycleGANCon step + VGG-19 content / Gram loss on fake_B2)
against tests/golden/c3_small.npz, which the REFERENCE CycleGANCon model with the reference
network.Vgg19 composed in produced (oracle/gen_golden_c3.py)."""
import numpy as np
import torch

from oracle import c3_ref, cpu_ref, prng, style_ref


def test_c3_step_matches_reference(golden):
    g = golden("c3_small")
    m = c3_ref.RefCycleGANConVGG(ngf=8, ndf=8)
    style_ref.load_np(m.vgg, style_ref.vgg_weights(m.vgg, 530))
    for name, seed in (("G_A", 1300), ("G_B", 1400), ("D_A", 1500), ("D_B", 1600)):
        net = m.nets()[name]
        cpu_ref.load_np_state(net, prng.init_state_dict(cpu_ref.state_shapes(net), base_seed=seed))
    m.set_input_fc2(*(torch.from_numpy(g[k]) for k in ("real_A", "real_A2", "real_B", "mask", "flow")))
    names = [str(n) for n in g["loss_names"]]
    assert names == m.loss_names
    for s in range(g["losses"].shape[0]):
        m.optimize_parameters()
        cur = m.get_current_losses()
        np.testing.assert_allclose([cur[n] for n in names], g["losses"][s], rtol=1e-4)
    with torch.no_grad():
        out = m.G_A(torch.from_numpy(g["probe"]))
    np.testing.assert_allclose(out.numpy(), g["probe_out"], rtol=1e-3, atol=1e-4)
