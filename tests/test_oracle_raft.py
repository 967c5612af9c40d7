"""Pin the RAFT oracle (oracle/raft_ref.py) against the reference RAFT's own outputs
(oracle/gen_golden_raft.py imported utils/raft/raft/raft.py).  CPU only."""
import numpy as np
import torch

from oracle import raft_ref


def _rel(got, ref):
    got, ref = np.asarray(got, np.float64), np.asarray(ref, np.float64)
    return np.abs(got - ref).max() / (np.abs(ref).max() + 1e-30)


def _sd(g):
    import argparse
    from gbvst import raft
    model = raft.RAFT(argparse.Namespace(small=False))
    shapes = {k: tuple(v.shape) for k, v in model.state_dict().items()}
    assert sorted(shapes) == list(g["keys"]), "module tree / state_dict keys differ from the reference RAFT"
    return {k: torch.from_numpy(np.asarray(v)) for k, v in raft_ref.raft_weights(shapes, 1300).items()}


def test_raft_oracle_matches_reference(golden):
    g = golden("raft_small")
    sd = _sd(g)
    pads = tuple(int(v) for v in g["pads"])
    assert pads == raft_ref.input_pads(g["img1"].shape)
    i1 = raft_ref.pad_replicate(torch.from_numpy(g["img1"]), pads)
    i2 = raft_ref.pad_replicate(torch.from_numpy(g["img2"]), pads)
    with torch.no_grad():
        (low, up), (f1, f2, c) = raft_ref.raft_forward(sd, i1, i2, iters=6, test_mode=True, with_features=True)
        preds = raft_ref.raft_forward(sd, i1, i2, iters=3, test_mode=False)
    assert _rel(f1, g["fmap1"]) < 1e-5 and _rel(f2, g["fmap2"]) < 1e-5
    assert _rel(c, g["cnet"]) < 1e-5
    assert _rel(low, g["low6"]) < 1e-4
    assert _rel(up, g["up6"]) < 1e-4
    assert _rel(torch.stack(preds), g["preds3"]) < 1e-4
