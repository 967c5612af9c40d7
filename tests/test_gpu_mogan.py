"""GPU parity of the MoGAN train step: gbvst.mogan_model against the reference
MoGAN model's own losses (tests/golden/mogan_small.npz: E-step then M-step, 1x3x128x128, ngf 8,
RAFT with 20 iterations and counter-PRNG weights).

Tolerances: step-1 losses 1e-3 relative (north_star; G/D/M forward at fp32-equivalent arithmetic,
RAFT 20 GRU iterations); the step-1 RAFT flow 1e-3 of max|flow|; the fb-check mask exact; step-2
(after one Adam update of G and D) 2e-3 relative."""
import argparse

import numpy as np
import pytest
import torch

from oracle import prng, raft_ref

pytestmark = pytest.mark.gpu
DEV = "cuda"
SEEDS = {"G_A": 1500, "G_B": 1501, "D_A": 1502, "D_B": 1503, "M_A": 1504, "M_B": 1505}


@pytest.fixture(scope="module")
def gb():
    import gbvst
    gbvst._lib.load()
    return gbvst


def _model():
    from gbvst import mogan_model, raft
    from gbvst.options import default_opt
    r = raft.RAFT(argparse.Namespace(small=False))
    shapes = {k: tuple(v.shape) for k, v in r.state_dict().items()}
    r.load_state_dict({k: torch.from_numpy(np.asarray(v)) for k, v in raft_ref.raft_weights(shapes, 1300, 1e-3).items()})
    r = r.to(DEV).eval()
    opt = default_opt(True, model="mogan", ngf=8, ndf=8, pool_size=0, gpu_ids=[0])
    m = mogan_model.MoGANModel(opt, raft_model=r)
    for name, seed in SEEDS.items():
        net = getattr(m, "net" + name)
        shapes = {k: tuple(v.shape) for k, v in net.state_dict().items()}
        net.load_state_dict({k: torch.from_numpy(v) for k, v in prng.init_state_dict(shapes, base_seed=seed).items()})
    return m


def test_mogan_steps_vs_reference_golden(gb, golden):
    g = golden("mogan_small")
    m = _model()
    names = list(g["loss_names"])
    imgs = [torch.from_numpy(g["img%d" % i]) for i in range(4)]
    for step in range(2):
        m.set_input_fc2(imgs)
        m.optimize_parameters()
        got = np.array([float(getattr(m, "loss_" + n)) if hasattr(m, "loss_" + n) else np.nan for n in names])
        ref = g["losses"][step]
        np.testing.assert_array_equal(np.isnan(got), np.isnan(ref))
        k = ~np.isnan(ref)
        np.testing.assert_allclose(got[k], ref[k], rtol=1e-3 if step == 0 else 2e-3, atol=1e-6,
                                   err_msg=f"step {step}")
        if step == 0:
            from gbvst import ops
            bf = ops.nhwc_to_nchw(m.bf_real_A, 2).cpu().numpy()
            assert np.abs(bf - g["bf_real_A"]).max() <= 1e-3 * np.abs(g["bf_real_A"]).max()
            assert np.array_equal(m.mask_A.cpu().numpy(), g["mask_A"])
    assert m.e_step  # E, M, back to E
