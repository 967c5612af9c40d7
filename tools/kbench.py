"""Developer: launch one conv family on the ResnetBlock shape (B=4, 64x64x256, 3x3 reflect) a few
times (batch KB_B, default 8) — the target of rocprofv3 --pmc passes.  usage: kbench.py fprop|dgrad|tconv|wgrad|wgrad_pre|wgrad_nhwc|warp|c0 [reps]
(wgrad_pre: the weight gradient as the train step runs it, on the IN passes' premade x image / dy planes)
warp: vst_warp_fwd on bench.py's warp_roofline shape (N=32, C=64, 436x1024, its smooth flow; KB_FLOW=iid:
the i.i.d. worst case).  c0: the generator's first conv (conv_c4_ring_k; VST_C4_RING=0: conv_c4_direct_k) at N=KB_B, 256x256."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import gbvst  # noqa: E402
from gbvst import ops  # noqa: E402

gbvst._lib.load()
which = sys.argv[1]
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 10
dev = torch.device("cuda")
if which == "warp":
    import torch.nn.functional as F
    N, C, H, W = 32, 64, 436, 1024
    xw = torch.randn(N, H, W, C, device=dev)
    if os.environ.get("KB_FLOW", "smooth") == "iid":
        flow = torch.randn(N, 2, H, W, device=dev) * 3.0
    else:  # bench.py warp_roofline's SURVEY 8d smooth flow (bicubic 9x9 N(0, 4^2) grid, x4)
        g = torch.Generator(device="cpu").manual_seed(4321)
        coarse = torch.randn(N, 2, 9, 9, generator=g) * 4.0
        flow = (F.interpolate(coarse, size=(H, W), mode="bicubic", align_corners=True) * 4.0).to(dev).contiguous()
    out = torch.empty_like(xw)
    for _ in range(reps):
        ops.lib().vst_warp_fwd(xw.data_ptr(), flow.data_ptr(), out.data_ptr(), N, H, W, C, 0,
                               torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    sys.exit(0)
if which == "c0":  # the generator's first conv (4-channel image -> 64, 7x7 reflect 3) with IN partials
    B = int(os.environ.get("KB_B", "8"))
    x4 = torch.rand(B, 256, 256, 4, device=dev) * 2 - 1
    x4[..., 3] = 0
    k0 = ops.weight_pack(torch.randn(64, 3, 7, 7, device=dev) * 0.05, ops.PACK_FWD)
    b0 = torch.zeros(64, device=dev)
    for _ in range(reps):
        ops.conv2d_fwd_in(x4, k0, b0, 64, 7, 7, 1, 3, "reflect")
    torch.cuda.synchronize()
    sys.exit(0)
B, H, C = int(os.environ.get("KB_B", "8")), 64, 256  # 8 = the batched G_A calls of the train step
x = torch.randn(B, H, H, C, device=dev)
# KB_RELU=1: x = relu(randn) (half zeros, as the step's post-IN/ReLU activations) — the operands' toggle rate sets
# the clock the chip holds under MFMA load (MI355X_MICROARCH.md DVFS items)
if os.environ.get("KB_RELU") == "1":
    x = torch.relu(x)
w = torch.randn(C, C, 3, 3, device=dev) * 0.02
kc, ck = ops.weight_pack(w, ops.PACK_FWD), ops.weight_pack(w, ops.PACK_DGRAD)
ikf = ops.weight_pack(w, ops.PACK_IKF)
gy = torch.randn(B, H, H, C, device=dev)
dw = torch.zeros(C, C, 3, 3, device=dev)
if which == "wgrad_pre":  # the step's form: x's padded image and dy's planes made by their producers
    st = torch.zeros((B, C, 2), device=dev)
    st[..., 1] = 1.0
    _, x_t = ops.instnorm_act_fwd(x, st, "none", cp=(1, "reflect", 1))
    gy, dy_planes = ops.instnorm_act_bwd(gy, x, st, "none", planes=True)
    torch.cuda.synchronize()
if which == "wgrad_nhwc":  # round 6: x NHWC itself, dy as its NHWC planes only (vst_conv2d_wgrad_nhwc)
    st = torch.zeros((B, C, 2), device=dev)
    st[..., 1] = 1.0
    gy = ops.instnorm_act_bwd(gy, x, st, "none", apre=True)
    torch.cuda.synchronize()
# KB_FLUSH=1: a 1 GiB write before every call (L2 and the MALL hold none of the operands: the cold-operand
# time); KB_FLUSH=2 (wgrad_pre): then the dy planes re-made by their producer (hot, as in the step; x's image cold)
flush = torch.empty(1 << 28, device=dev) if os.environ.get("KB_FLUSH") else None
for _ in range(reps):
    if flush is not None:
        flush.fill_(1.0)
        if which == "wgrad_pre" and os.environ.get("KB_FLUSH") == "2":
            gy, dy_planes = ops.instnorm_act_bwd(gy, x, st, "none", planes=True)
    if which == "fprop":
        ops.conv2d_fwd(x, kc, None, C, 3, 3, 1, 1, "reflect")
    elif which == "dgrad":  # stride-1 data gradient as a forward conv over rotated taps (train path)
        ops.conv2d_dgrad_s1(gy, ikf, H, H, C, 3, 1, "reflect")
    elif which == "tconv":
        ops.conv2d_tfwd(gy, ck, None, H, H, C, 3, 3, 1, 1, pad_mode="reflect")
    elif which == "wgrad_pre":
        ops.conv2d_wgrad(x, gy, dw, None, 3, 3, 1, 1, "reflect", C, C, C * 9, 9, dy_planes=dy_planes, x_t=x_t)
    else:
        ops.conv2d_wgrad(x, gy, dw, None, 3, 3, 1, 1, "reflect", C, C, C * 9, 9)
torch.cuda.synchronize()
