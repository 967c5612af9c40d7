"""Pin the CPU oracle (oracle/cpu_ref.py) against golden vectors produced by the reference itself
(oracle/gen_golden.py imported /root/reference in the build container)."""
import numpy as np
import torch

from oracle import cpu_ref, prng


def test_prng_known_answer(golden):
    g = golden("prng")
    np.testing.assert_array_equal(prng.uniform(7, 16), g["u"])
    np.testing.assert_array_equal(prng.normal(7, (17,)), g["n"])


def test_warp_matches_reference(golden):
    g = golden("warp")
    for case in ("zero", "int", "frac", "oob", "h1", "w1"):
        x = torch.from_numpy(g[f"{case}_x"]).requires_grad_(True)
        y = cpu_ref.warp(x, torch.from_numpy(g[f"{case}_flow"]))
        y.backward(torch.from_numpy(g[f"{case}_gout"]))
        np.testing.assert_allclose(y.detach().numpy(), g[f"{case}_y"], rtol=0, atol=1e-6)
        np.testing.assert_allclose(x.grad.numpy(), g[f"{case}_dx"], rtol=0, atol=1e-6)


def test_fbc_matches_reference(golden):
    g = golden("fbc")
    for case in ("cons", "incons"):
        m = cpu_ref.fbc_check(torch.from_numpy(g[f"{case}_ff"]), torch.from_numpy(g[f"{case}_bf"]))
        np.testing.assert_array_equal(m.numpy(), g[f"{case}_mask"])
    assert 0 < g["incons_mask"].mean() < 1


def _check_net(g, tag, net):
    sd = {k[len(tag) + 3:]: g[k] for k in g.files if k.startswith(f"{tag}_w_")}
    cpu_ref.load_np_state(net, sd)
    x = torch.from_numpy(g[f"{tag}_x"]).requires_grad_(True)
    y = net(x)
    y.backward(torch.from_numpy(g[f"{tag}_gy"]))
    np.testing.assert_allclose(y.detach().numpy(), g[f"{tag}_y"], rtol=1e-5, atol=1e-5)
    np.testing.assert_allclose(x.grad.numpy(), g[f"{tag}_dx"], rtol=1e-4, atol=1e-5)
    for k, p in net.named_parameters():
        ref = g[f"{tag}_g_{k}"]
        scale = max(np.abs(ref).max(), 1e-6)
        assert np.abs(p.grad.numpy() - ref).max() / scale < 1e-4, k


def test_generator_matches_reference(golden):
    _check_net(golden("nets_small"), "G", cpu_ref.RefResnetGenerator(3, 3, 8, 9))


def test_discriminator_matches_reference(golden):
    _check_net(golden("nets_small"), "D", cpu_ref.RefNLayerDiscriminator(3, 8))


def test_train_step_matches_reference(golden):
    g = golden("step_small")
    m = cpu_ref.RefCycleGANCon(ngf=8, ndf=8)
    for name, net in m.nets().items():
        pre = f"w_{name}_"
        cpu_ref.load_np_state(net, {k[len(pre):]: g[k] for k in g.files if k.startswith(pre)})
    m.set_input_fc2(*(torch.from_numpy(g[k]) for k in ("real_A", "real_A2", "real_B", "mask", "flow")))
    names = [str(n) for n in g["loss_names"]]
    for s in range(g["losses"].shape[0]):
        m.optimize_parameters()
        cur = m.get_current_losses()
        np.testing.assert_allclose([cur[n] for n in names], g["losses"][s], rtol=1e-4)
    with torch.no_grad():
        out = m.G_A(torch.from_numpy(g["probe"]))
    np.testing.assert_allclose(out.numpy(), g["probe_out"], rtol=1e-3, atol=1e-4)


def test_ordered_warp_backward_matches_reference(golden):
    """oracle/flow_ref.warp_bwd_ordered (the deterministic warp backward's checker) against the
    reference's own grid_sample input gradients: same corner weights, only the summation order of
    colliding contributions differs (the align_corners=False quirk makes even integer flows sample
    between pixels, so every case has collisions)."""
    from oracle import flow_ref
    g = golden("warp")
    for case in ("zero", "int", "frac", "oob", "h1", "w1"):
        gout = np.ascontiguousarray(g[f"{case}_gout"].transpose(0, 2, 3, 1))
        dx = flow_ref.warp_bwd_ordered(gout, g[f"{case}_flow"]).transpose(0, 3, 1, 2)
        np.testing.assert_allclose(dx, g[f"{case}_dx"], rtol=0, atol=1e-6)
    # the masked variant (fs_lib.warp) and align_corners=True against torch autograd on CPU
    x = torch.from_numpy(prng.uniform_f32(71, (2, 4, 9, 11), -1.0, 1.0)).requires_grad_(True)
    fl = torch.from_numpy(prng.normal(72, (2, 2, 9, 11), std=2.0).astype(np.float32))
    go = torch.from_numpy(prng.uniform_f32(73, (2, 4, 9, 11), -1.0, 1.0))
    for align in (False, True):
        x.grad = None
        cpu_ref.warp(x, fl, align_corners=align).backward(go)
        dx = flow_ref.warp_bwd_ordered(go.permute(0, 2, 3, 1).numpy(), fl.numpy(), align=align)
        np.testing.assert_allclose(dx.transpose(0, 3, 1, 2), x.grad.numpy(), rtol=0, atol=2e-6)
