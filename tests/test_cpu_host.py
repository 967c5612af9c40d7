"""CPU-only checks: the C-ABI library exports every symbol include/vst_hip.h declares, the host
logic (state_dict compatibility with the reference, options, plugin discovery) matches the
reference, and the product path refuses CPU tensors (no silent fallback)."""
import ctypes
import os
import re

import pytest
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _header_symbols():
    txt = open(os.path.join(REPO, "include", "vst_hip.h")).read()
    return sorted(set(re.findall(r"^\s*(?:const\s+)?\w+\*?\s+\**(vst_\w+)\(", txt, re.M)))


def test_library_exports_every_header_symbol():
    import gbvst
    path = gbvst._lib.build()
    lib = ctypes.CDLL(path)
    syms = _header_symbols()
    assert len(syms) >= 25
    for s in syms:
        assert hasattr(lib, s), s
    assert set(syms) == set(gbvst._lib.SIGNATURES), set(syms) ^ set(gbvst._lib.SIGNATURES)


def test_state_dict_matches_reference_layout():
    from gbvst import networks
    from oracle import cpu_ref
    for ngf, nb in ((64, 9), (8, 6)):
        G = networks.define_G(3, 3, ngf, "resnet_%dblocks" % nb, "instance", False, "normal", 0.02, [])
        R = cpu_ref.RefResnetGenerator(3, 3, ngf, nb)
        assert cpu_ref.state_shapes(G) == cpu_ref.state_shapes(R)
    D = networks.define_D(3, 64, "basic", 3, "instance", "normal", 0.02, [])
    assert cpu_ref.state_shapes(D) == cpu_ref.state_shapes(cpu_ref.RefNLayerDiscriminator(3, 64))
    assert sum(p.numel() for p in G.parameters()) > 0


def test_flat_buffers_are_views():
    from gbvst import networks
    G = networks.define_G(3, 3, 8, "resnet_9blocks", "instance", False, "normal", 0.02, [])
    n = sum(p.numel() for p in G.parameters())
    assert G.flat_param.numel() == n
    with torch.no_grad():
        G.flat_param.fill_(0.5)
    assert all(float(p.detach().mean()) == 0.5 for p in G.parameters())
    sd = {k: torch.full_like(v, 0.25) for k, v in G.state_dict().items()}
    G.load_state_dict(sd)
    assert float(G.flat_param.mean()) == 0.25


def test_unsupported_configs_raise():
    from gbvst import networks
    with pytest.raises(NotImplementedError):
        networks.define_G(3, 3, 64, "unet_256", "instance")
    with pytest.raises(NotImplementedError):
        networks.define_G(3, 3, 64, "nope", "instance")
    with pytest.raises(NotImplementedError):
        networks.get_norm_layer("group")


def test_options_and_plugin_discovery():
    from gbvst import models, options
    opt = options.default_opt(True)
    for k, v in dict(ngf=64, ndf=64, netG="resnet_9blocks", netD="basic", norm="instance",
                     init_gain=0.02, lr=2e-4, beta1=0.5, gan_mode="lsgan", pool_size=50,
                     lr_policy="linear", n_epochs=100, n_epochs_decay=100, lambda_A=10.0,
                     lambda_B=10.0, lambda_T=10.0, lambda_identity=0.5).items():
        assert getattr(opt, k) == v, k
    assert opt.gpu_ids == [0]
    assert models.find_model_using_name("cycle_gan").__name__ == "CycleGANModel"
    with pytest.raises(NotImplementedError):
        models.find_model_using_name("pix2pix")


def test_ops_refuse_cpu_tensors():
    from gbvst import ops
    with pytest.raises(RuntimeError):
        ops.nchw_to_nhwc(torch.zeros(1, 3, 4, 4))


def test_style_modules_match_reference_layout():
    """FastStyleNet / Vgg16 / Vgg19 keep network.py's module tree: identical state_dict keys and
    shapes (reference checkpoints load by name), 1,679,240 FastStyleNet(3, 1) parameters."""
    from gbvst import faststyle, perceptual
    from oracle import style_ref
    n = faststyle.FastStyleNet(3, 1)
    assert cpu_state(n) == cpu_state(style_ref.RefFastStyleNet(3))
    assert sum(p.numel() for p in n.parameters()) == 1679240
    assert cpu_state(perceptual.Vgg16()) == cpu_state(style_ref.RefVGG("vgg16"))
    assert cpu_state(perceptual.Vgg19()) == cpu_state(style_ref.RefVGG("vgg19"))
    with pytest.raises(NotImplementedError):
        faststyle.FastStyleNet(3, n_styles=2)


def cpu_state(net):
    return {k: tuple(v.shape) for k, v in net.state_dict().items()}


def test_stargan_modules_match_reference_layout():
    """Generator / Discriminator keep StarGAN/model.py's module tree (state_dict keys, shapes and the
    InstanceNorm running buffers), at the solver defaults and at the fixture config."""
    from gbvst import stargan
    from oracle import stargan_ref
    for args in ((64, 5, 6), (8, 4, 2)):
        assert cpu_state(stargan.Generator(*args)) == cpu_state(stargan_ref.RefGenerator(*args))
    for args in ((128, 64, 5, 6), (256, 64, 4, 6), (32, 8, 4, 4)):
        assert cpu_state(stargan.Discriminator(*args)) == cpu_state(stargan_ref.RefDiscriminator(*args))
    d = stargan.Discriminator(256, 64, 4, 6)
    assert d.k == 4 and d.conv2.weight.shape == (4, 2048, 4, 4)
    oh = stargan.label2onehot(torch.tensor([2, 0]), 4, "cpu")
    assert oh.tolist() == [[0, 0, 1, 0], [1, 0, 0, 0]]


def test_raft_module_tree_and_no_cpu_fallback():
    """gbvst.raft.RAFT keeps raft.py's state_dict keys (checked against the reference list in
    tests/golden/raft_small.npz) and refuses to run on CPU tensors (no fallback path)."""
    import argparse

    import numpy as np
    from gbvst import raft
    m = raft.RAFT(argparse.Namespace(small=False))
    g = np.load(os.path.join(os.path.dirname(__file__), "golden", "raft_small.npz"), allow_pickle=False)
    assert sorted(m.state_dict()) == list(g["keys"])
    assert m.args.corr_levels == 4 and m.args.corr_radius == 4
    with pytest.raises(NotImplementedError):
        raft.RAFT(argparse.Namespace(small=True))
    assert raft.InputPadder((1, 3, 436, 1024)).pads == (0, 0, 2, 2)
    assert raft.InputPadder((1, 3, 436, 1024), mode="kitti").pads == (0, 0, 0, 4)
    x = torch.zeros(1, 3, 64, 64)
    with pytest.raises(RuntimeError):
        m(x, x, iters=1, test_mode=True)


def test_conv_planner_picks_production_kernels():
    """The host planner (vst_conv_plan_fwd, no device needed) routes the train step's dominant
    shapes to the kernels the GPU parity tests force and check: the N=8 ResnetBlock forward under
    bf16x6 -> 256x128 tiles (kind 7, one launch); its stride-1 data gradient over the padded frame
    (66x66, zero pad 2) under bf16x3 -> 128x128 tiles + a 64x64 wave-quantisation tail launch
    (546 = 2 x 256 + 34 blocks); fp32 -> the [row][k] kernel; 4 output channels -> VALU."""
    import gbvst
    from gbvst import ops
    gbvst._lib.load()
    assert ops.conv_plan_fwd(8, 64, 64, 256, 256, 3, 3, 1, 1, 1, "bf16x6") == (7, 0)
    # bf16x6 padded-frame dgrad (274 256x128 tiles): one whole round + a 64x64 tail launch
    assert ops.conv_plan_fwd(8, 64, 64, 256, 256, 3, 3, 1, 2, 2, "bf16x6", with_tail=True) == (7, 32768, 8)
    kind, ms = ops.conv_plan_fwd(8, 64, 64, 256, 256, 3, 3, 1, 2, 2, "bf16x3")
    assert kind == 0 and ms == 2 * 256 // 2 * 128 and 0 < ms < 8 * 66 * 66
    assert ops.conv_plan_fwd(8, 64, 64, 256, 256, 3, 3, 1, 1, 1, "fp32") == (ops.PLAN_RK, 0)
    assert ops.conv_plan_fwd(2, 32, 32, 64, 4, 7, 7, 1, 3, 3, "bf16x6")[0] == ops.PLAN_SKINNY
    # the generator's first conv: a 4-channel image on the split-bf16 kernels (not the fp32 rk path)
    assert ops.conv_plan_fwd(8, 256, 256, 4, 64, 7, 7, 1, 3, 3, "bf16x6")[0] not in (ops.PLAN_RK, ops.PLAN_SKINNY)
    assert ops.conv_plan_fwd(8, 256, 256, 4, 64, 7, 7, 1, 3, 3, "fp32")[0] == ops.PLAN_RK
    # 4 channels -> 64 at stride 1 (the generator's c0 at 256^2 and at Sintel width, a zero-pad-6 frame,
    # a short row): the patch-staged direct kernel; not where a row would end in a short extra
    # segment (the last layer's 262-wide data-gradient frame), nor where its InstanceNorm partials could
    # not follow the 32-pixel groups (H*W % 32 == 0 but Wo % 32 != 0), nor under a forced tile
    for shp in [(8, 256, 256, 3), (1, 436, 1024, 3), (8, 250, 250, 6), (2, 20, 18, 3)]:
        N_, H_, W_, p_ = shp
        for m_ in ("bf16x6", "bf16x3"):
            assert ops.conv_plan_fwd(N_, H_, W_, 4, 64, 7, 7, 1, p_, p_, m_)[0] == ops.PLAN_C4_DIRECT, (shp, m_)
    assert ops.conv_plan_fwd(2, 8, 8, 4, 64, 7, 7, 1, 3, 3, "bf16x6")[0] != ops.PLAN_C4_DIRECT
    assert ops.conv_plan_fwd(8, 256, 256, 4, 64, 7, 7, 1, 6, 6, "bf16x6")[0] != ops.PLAN_C4_DIRECT
    assert ops.conv_plan_fwd(2, 32, 32, 4, 64, 4, 4, 2, 1, 1, "bf16x6")[0] != ops.PLAN_C4_DIRECT
    assert ops.conv_plan_fwd(2, 32, 32, 4, 32, 7, 7, 1, 3, 3, "bf16x6")[0] != ops.PLAN_C4_DIRECT
    ops.debug_set_tiles(1, -1, -1)
    try:
        assert ops.conv_plan_fwd(8, 256, 256, 4, 64, 7, 7, 1, 3, 3, "bf16x6")[0] == 1
    finally:
        ops.debug_set_tiles(-1, -1, -1)
    ops.debug_set_tiles(7, -1, -1)
    try:
        assert ops.conv_plan_fwd(2, 12, 10, 32, 32, 3, 3, 1, 1, 1, "bf16x3") == (7, 0)
        # the override is thread-local: another host thread still plans automatically
        import threading
        out = []
        t = threading.Thread(target=lambda: out.append(ops.conv_plan_fwd(2, 12, 10, 32, 32, 3, 3, 1, 1, 1, "bf16x3")))
        t.start()
        t.join()
        assert out[0][0] != 7
    finally:
        ops.debug_set_tiles(-1, -1, -1)


def test_pack_batch_records_match_the_abi_layout():
    """ops.PackBatch job records: 168 bytes each, the field order of include/vst_hip.h's
    vst_weight_pack_batch record (and misc.hip's static_assert on sizeof(PackJob))."""
    import re
    import struct
    from gbvst import ops
    assert struct.calcsize("<3Q8i2q4q8i8i") == ops.PackBatch.REC == 168
    hdr = open(os.path.join(REPO, "include", "vst_hip.h")).read()
    assert "168-byte records" in hdr and "int vst_weight_pack_batch(const void* jobs" in hdr
    src = open(os.path.join(REPO, "gan-based-video-style-transfer_amd", "csrc", "misc.hip")).read()
    assert re.search(r"static_assert\(sizeof\(PackJob\) == 168", src)


def test_wgrad_planner_routes_generator_layers_to_bf16_kernel():
    """Host-only vst_conv_plan_wgrad: under bf16x6 every generator weight gradient of the C2 step
    (incl. the 8-channel image edge and the stride-2 layers) runs the split-bf16 kernel
    conv_wgrad_bf_k; the ResnetBlock one on 256x128 tiles (kind 7) in 14 split-K slabs."""
    import gbvst
    from gbvst import ops
    gbvst._lib.load()
    BF = 2
    shapes = {  # N, H, W, Cx, Ho, Wo, Cyp, R, S, stride
        "c0": (8, 256, 256, 8, 256, 256, 64, 7, 7, 1), "d0": (8, 256, 256, 64, 128, 128, 128, 3, 3, 2),
        "d1": (8, 128, 128, 128, 64, 64, 256, 3, 3, 2), "res": (8, 64, 64, 256, 64, 64, 256, 3, 3, 1),
        "u0": (8, 128, 128, 128, 64, 64, 256, 3, 3, 2), "u1": (8, 256, 256, 64, 128, 128, 128, 3, 3, 2),
        "D0": (8, 256, 256, 4, 128, 128, 64, 4, 4, 2)}
    for name, sh in shapes.items():
        path, kind, ns = ops.conv_plan_wgrad(*sh, "bf16x6")
        assert path == BF, (name, path)
    assert ops.conv_plan_wgrad(*shapes["res"], "bf16x6")[1:] == (7, 14)


def test_wrong_result_modes_refused_in_product_build():
    """VERDICT r2 hygiene: the developer timing modes of conv_bf.hip that compute wrong results
    (VST_BF_FAKESPLIT, VST_BF_FAKE16) stop the preprocessor unless the variant builder's
    VST_DEV_VARIANT is defined; the product builder refuses that define."""
    import subprocess
    import pytest
    from gbvst import _lib
    src = os.path.join(_lib.CSRC, "conv_bf.hip")
    for mode in ("VST_BF_FAKESPLIT=1", "VST_BF_FAKE16=1", "VST_BF_FAKE_ZA=1", "VST_BF_FAKE_ZB=1"):
        r = subprocess.run([_lib.HIPCC, "-E", "--offload-arch=gfx950", "--cuda-host-only", "-D" + mode, src,
                            "-o", os.devnull], stdout=subprocess.PIPE, stderr=subprocess.STDOUT)
        assert r.returncode != 0 and b"developer-only" in r.stdout, (mode, r.stdout[-400:])
    r = subprocess.run([_lib.HIPCC, "-E", "--offload-arch=gfx950", "--cuda-host-only", "-DVST_BF_FAKESPLIT=1",
                        "-DVST_DEV_VARIANT=1", src, "-o", os.devnull], stdout=subprocess.PIPE, stderr=subprocess.STDOUT)
    assert r.returncode == 0, r.stdout[-400:]
    with pytest.raises(ValueError):
        _lib.build(defines=["VST_DEV_VARIANT=1"])


def test_conv_desc_host_validation():
    """§8b descriptor entry points validate on the host before any launch (no GPU needed)."""
    import ctypes
    import gbvst
    lib = gbvst._lib.load()
    d = gbvst._lib.VstConvDesc()
    for k, v in dict(N=2, H=64, W=64, C=256, K=256, R=3, S=3, stride=1, pad=1, pad_mode=1, dilation=1,
                     math=2).items():
        setattr(d, k, v)
    ho, wo = ctypes.c_int(), ctypes.c_int()
    assert lib.vst_conv_desc_out_hw(ctypes.byref(d), ctypes.byref(ho), ctypes.byref(wo)) == 0
    assert (ho.value, wo.value) == (64, 64)
    assert lib.vst_workspace_size(ctypes.byref(d), 2) == lib.vst_conv2d_wgrad_ws_bytes(2, 64, 64, 256, 64, 64, 256,
                                                                                      3, 3, 1)
    d.transposed, d.pad_mode, d.stride, d.output_padding, d.H, d.W = 1, 0, 2, 1, 32, 32
    assert lib.vst_conv_desc_out_hw(ctypes.byref(d), ctypes.byref(ho), ctypes.byref(wo)) == 0
    assert (ho.value, wo.value) == (64, 64)
    for field, bad in (("dilation", 2), ("layout", 1), ("dtype", 3), ("C", 6), ("output_padding", 2)):
        old = getattr(d, field)
        setattr(d, field, bad)
        assert lib.vst_conv_desc_out_hw(ctypes.byref(d), ctypes.byref(ho), ctypes.byref(wo)) == 1, field
        assert lib.vst_workspace_size(ctypes.byref(d), 0) == 0
        setattr(d, field, old)
    assert lib.vst_conv_desc_out_hw(None, ctypes.byref(ho), ctypes.byref(wo)) == 1


def test_convflops_counter_wraps_live_ops():
    """bench.py's FLOP counter (tools/convflops.Counter) wraps ops functions by name: every name it lists must
    exist in gbvst.ops (a route deleted from ops must leave the counter too, or bench.py fails on the box)."""
    import sys
    sys.path.insert(0, os.path.join(REPO, "tools"))
    import convflops
    from gbvst import ops
    missing = [n for n in convflops.OPS if not hasattr(ops, n)]
    assert not missing, missing
    with convflops.Counter():
        pass
