"""TEST INFRASTRUCTURE ONLY — the CPU oracle for the CycleGAN video train-step hot path.

Nothing in the product package (`gan-based-video-style-transfer_amd/`) imports this package.
Only `tests/`, `__graft_entry__.smoke()` and `bench.py`'s `cpu_baseline` leg may import it, and
only as the checker / the timed CPU baseline, never as the thing measured or shipped.

Contents
  prng.py      portable counter-based PRNG (splitmix64 -> uniform -> Box-Muller); used to
               generate identical weights/inputs for the reference, the oracle and the HIP path.
  cpu_ref.py   stock-PyTorch-CPU (NCHW fp32) restatement of the reference hot path
               (ResnetGenerator, NLayerDiscriminator, flow warp, fb-check, losses, the
               CycleGANCon optimize_parameters step, forward_eval). Every function cites the
               reference file:line it restates.
  gen_golden.py  run in the build container only: imports the read-only reference and writes
               the golden fixtures under tests/golden/ (inputs + reference outputs).

Parity pinning: the reference is pure Python/PyTorch, so the oracle is pinned against golden
vectors produced by importing the reference itself in this container.
"""
