"""TEST INFRASTRUCTURE ONLY: CountSketch of a tensor, the compact stand-in for a full-size oracle gradient
in the committed fixtures (tests/golden/fullsize_*.npz, oracle/gen_fullsize_refs.py).

Element i of the flattened tensor goes to bucket b(i) with sign s(i) (integer hashes of i, identical on
CPU and GPU); sketch[b] = sum s(i) v_i.  For the difference of two tensors, E ||CS(u) - CS(v)||^2 =
||u - v||^2, with a relative standard error of ~sqrt(2 / K) on the squared norm (K = 1024: the norm
to ~2-3 %), so a norm-wise deviation ||HIP - ref|| / ||ref|| is measured from the sketches alone.
"""
import torch

K = 1024


def count_sketch(v, k=K):
    v = torch.as_tensor(v).reshape(-1).double()
    i = torch.arange(v.numel(), device=v.device, dtype=torch.int64)
    b = ((i * 2654435761) >> 11) % k          # < 2^63 for every index below 3e9
    s = (((i * 2246822507) >> 17) & 1) * 2 - 1
    out = torch.zeros(k, dtype=torch.float64, device=v.device)
    out.index_add_(0, b, v * s.double())
    return out


def sketch_dev(cs_got, cs_ref, ref_norm):
    """Estimated ||got - ref|| / ||ref|| from the two sketches and the exact ||ref||."""
    d = torch.as_tensor(cs_got).double().cpu() - torch.as_tensor(cs_ref).double().cpu()
    return float(d.norm() / (ref_norm + 1e-300))
