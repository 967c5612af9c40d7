"""Pin the MoGAN step oracle (oracle/mogan_ref.py) against the reference MoGAN model's own losses
(oracle/gen_golden_mogan.py ran methods/GAN-based/MoGAN/models/cycle_gan_model.py).  CPU only."""
import numpy as np
import torch

from oracle import cpu_ref, mogan_ref, prng, raft_ref

SEEDS = {"G_A": 1500, "G_B": 1501, "D_A": 1502, "D_B": 1503, "M_A": 1504, "M_B": 1505}


def raft_state(keys):
    import argparse
    from gbvst import raft
    shapes = {k: tuple(v.shape) for k, v in raft.RAFT(argparse.Namespace(small=False)).state_dict().items()}
    return raft_ref.raft_weights(shapes, 1300, 1e-3)


def test_mogan_oracle_matches_reference(golden):
    g = golden("mogan_small")
    sd = {k: torch.from_numpy(np.asarray(v)) for k, v in raft_state(None).items()}
    m = mogan_ref.RefMoGAN(sd, ngf=8, ndf=8)
    for name, net in m.nets().items():
        cpu_ref.load_np_state(net, prng.init_state_dict(cpu_ref.state_shapes(net), base_seed=SEEDS[name]))
    imgs = [torch.from_numpy(g["img%d" % i]) for i in range(4)]
    names = list(g["loss_names"])
    for step in range(2):
        m.set_input_fc2(*imgs)
        m.optimize_parameters()
        ls = m.get_current_losses()
        got = np.array([ls.get(n, np.nan) for n in names])
        np.testing.assert_allclose(got, g["losses"][step], rtol=1e-4, atol=1e-6, err_msg=f"step {step}")
        if step == 0:
            assert np.abs(m.bf_real_A.numpy() - g["bf_real_A"]).max() < 1e-4 * np.abs(g["bf_real_A"]).max() + 1e-7
            assert np.array_equal(m.mask_A.numpy(), g["mask_A"])
