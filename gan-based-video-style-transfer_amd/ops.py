"""Tensor-level wrappers over the C ABI (include/vst_hip.h).

Every function launches on torch's current HIP stream, takes/returns torch tensors that live on the
GPU, and raises on a non-zero status.  Activations are NHWC fp32 with a channel stride that is a
multiple of 4 (``cpad``); images are NHWC4.  There is no CPU fallback: a CPU tensor is an error.
"""
import functools
import os

import torch

from . import _lib

ACT = {"none": 0, "relu": 1, "lrelu": 2, "tanh": 3}
PAD = {"zero": 0, "reflect": 1}
PACK_KC, PACK_CK, PACK_OK, PACK_IK, PACK_IKF, PACK_SOK = 0, 1, 2, 3, 4, 5
# the conv kernels consume: forward conv -> PACK_OK, data-gradient / transposed conv -> PACK_IK
PACK_FWD, PACK_DGRAD = PACK_OK, PACK_IK
EUNSUPPORTED = 2  # VST_EUNSUPPORTED (include/vst_hip.h)
IN_EPS = 1e-5


def cpad(c):
    return (c + 3) // 4 * 4


def lib():
    return _lib.load()


def _stream():
    return torch.cuda.current_stream().cuda_stream


def _p(t):
    return None if t is None else t.data_ptr()


def _dev_check(*ts):
    for t in ts:
        if t is not None:
            if not t.is_cuda:
                raise RuntimeError("vst ops require GPU tensors (no CPU fallback)")
            if t.dtype != torch.float32 or not t.is_contiguous():
                raise RuntimeError("vst ops require contiguous float32 tensors")


def _call(name, *args):
    rc = getattr(lib(), name)(*args)
    if rc != 0:
        _lib.check(rc, name)


# ------------------------------------------------------------------------------------ layout
def nchw_to_nhwc(x, cs=None):
    _dev_check(x)
    N, C, H, W = x.shape
    cs = cs or cpad(C)
    y = torch.empty((N, H, W, cs), device=x.device, dtype=torch.float32)
    _call("vst_nchw_to_nhwc", _p(x), _p(y), N, C, H, W, cs, _stream())
    return y


def nhwc_to_nchw(x, c):
    _dev_check(x)
    N, H, W, cs = x.shape
    y = torch.empty((N, c, H, W), device=x.device, dtype=torch.float32)
    _call("vst_nhwc_to_nchw", _p(x), _p(y), N, c, H, W, cs, _stream())
    return y


def _pack_shape(mode, O, I_, R, S, Op=None, Ip=None):
    Op, Ip = Op or cpad(O), Ip or cpad(I_)
    return {PACK_KC: (R, S, Ip, Op), PACK_CK: (R, S, Op, Ip), PACK_OK: (Op, R, S, Ip),
            PACK_IK: (Ip, R, S, Op), PACK_IKF: (Ip, R, S, Op), PACK_SOK: (S * Op, R, 1, Ip)}[mode]


class PackBatch:
    """A network's weight packs as ONE launch (vst_weight_pack_batch).  Inside ``with PackBatch()``
    every weight_pack / convT3s2_phase_packs call allocates its outputs and records a job instead of
    launching; leaving the block packs them all.  ``run()`` re-packs every recorded job in place
    from the (updated) weights — after an optimizer step the pack set is refreshed by one kernel
    instead of one launch per pack.  The job sources are the live parameter tensors (views into the
    network's flat buffer), so the outputs stay valid objects across refreshes."""
    _active = None
    REC = 168  # sizeof(PackJob), include/vst_hip.h

    def __init__(self):
        self.jobs, self.blocks, self.copies, self._dev = [], 0, [], None

    def __enter__(self):
        self._prev, PackBatch._active = PackBatch._active, self
        return self

    def __exit__(self, *exc):
        PackBatch._active = self._prev
        if exc[0] is None and self.jobs:
            self.run()
        return False

    def add(self, w, mode, O, I_, R, S, strides, tr=None, ts=None, Op=None, Ip=None):
        import struct
        Op, Ip = Op or cpad(O), Ip or cpad(I_)
        shape = _pack_shape(mode, O, I_, R, S, Op, Ip)
        out = torch.empty(shape, device=w.device, dtype=torch.float32)
        split = torch.empty((3,) + shape, device=w.device, dtype=torch.bfloat16)
        out.vst_split = split
        total = out.numel()
        tr = list(tr) if tr is not None else [-1]  # -1: identity tap map (any R / S)
        ts = list(ts) if ts is not None else [-1]
        if len(tr) > 8 or len(ts) > 8:
            raise ValueError("PackBatch: explicit tap maps need R, S <= 8")
        rec = struct.pack("<3Q8i2q4q8i8i", w.data_ptr(), out.data_ptr(), split.data_ptr(), O, I_, R, S,
                          Op, Ip, mode, 0, total, self.blocks, *strides,
                          *(tr + [0] * (8 - len(tr))), *(ts + [0] * (8 - len(ts))))
        self.jobs.append((rec, w, out, split))
        self.blocks += (total + 255) // 256
        self._dev = None
        return out

    def copy_into(self, dst, src):
        """dst[:n] = src on every run (padded bias vectors)."""
        self.copies.append((dst, src))
        dst[:src.numel()].copy_(src)

    def run(self):
        if self._dev is None:
            buf = b"".join(j[0] for j in self.jobs)
            self._dev = torch.frombuffer(bytearray(buf), dtype=torch.uint8).to(self.jobs[0][1].device)
        _call("vst_weight_pack_batch", _p(self._dev), len(self.jobs), self.blocks, _stream())
        for dst, src in self.copies:
            dst[:src.numel()].copy_(src)


def weight_pack(w, mode, transposed=False, Op=None, Ip=None):
    """Pack a PyTorch conv weight for the GEMM kernels (see vst_weight_pack).  For a
    ConvTranspose2d weight [Ci][Co][R][S] pass transposed=True: dims are then (O=Ci, I=Co).
    Op / Ip: padded channel counts (default cpad; 8 lets a 3-channel side use the split-bf16
    kernels, whose K chunks are 8 channels deep)."""
    _dev_check(w)
    O, I_, R, S = w.shape
    Op, Ip = Op or cpad(O), Ip or cpad(I_)
    pb = PackBatch._active
    if pb is not None:
        return pb.add(w, mode, O, I_, R, S, (I_ * R * S, R * S, S, 1), Op=Op, Ip=Ip)
    shape = _pack_shape(mode, O, I_, R, S, Op, Ip)
    out = torch.empty(shape, device=w.device, dtype=torch.float32)
    # the split-arithmetic conv paths read the pack as three bf16 planes (written in the same pass)
    split = torch.empty((3,) + shape, device=w.device, dtype=torch.bfloat16)
    _call("vst_weight_pack_split", _p(w), _p(out), _p(split), O, I_, R, S, Op, Ip, mode, _stream())
    out.vst_split = split
    return out


# --------------------------------------------------------------------------------------- conv
class LaunchProbe:
    """Measurement hook (bench.py): HIP events around the launches of one conv op ("fwd" =
    vst_conv2d_fwd, "wgrad" = vst_conv2d_wgrad) of one shape (N, H, W, Cx, Cop, R, stride, pad,
    pad_mode), recorded on the stream the op is launched on.  every: events around one matching launch in
    `every` (`seen` counts them all) — an event pair costs the stream a few microseconds of idle time between
    kernels, so timing all 108 probed launches of a C2 step would add ~1 ms to the very step being measured;
    a stride coprime to the per-step launch count (36) samples every launch position over the steps."""

    def __init__(self, key, every=1):
        self.key, self.events, self.steps, self.every, self.seen = key, [], 1, max(1, int(every)), 0

    def mean_ms(self):
        torch.cuda.synchronize()
        t = [a.elapsed_time(b) for a, b in self.events]
        return sum(t) / len(t) if t else float("nan")


_probes = []


def set_launch_probes(probes):
    global _probes
    _probes = list(probes)


def _probe_begin(op, key):
    for p in _probes:
        if p.key == (op, key):
            p.seen += 1
            if (p.seen - 1) % p.every:
                return None
            ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
            ev[0].record()
            return p, ev
    return None


def _probe_end(h):
    if h is not None:
        p, ev = h
        ev[1].record()
        p.events.append(ev)


# Split-K tails of x6 forward grids (vst_conv2d_fwd_ws); False keeps the small-tile tails.  (Module flags
# like this one are route selectors the tests flip in-process to compare routes; they are not read from the
# environment.)
FWD_SPLITK = True
_fws_cache = {}


def _fwd_ws(N, H, W, Cx, cop, R, S, stride, pad, m, device):
    """Workspace tensor of vst_conv2d_fwd_ws for this shape (None when the launch needs none)."""
    if not FWD_SPLITK:
        return None, 0
    key = (N, H, W, Cx, cop, R, S, stride, pad, m)
    nb = _fws_cache.get(key)
    if nb is None:
        nb = _fws_cache[key] = int(lib().vst_conv2d_fwd_ws_bytes(N, H, W, Cx, cop, R, S, stride, pad, m))
    if nb == 0:
        return None, 0
    return torch.empty((nb + 3) // 4, device=device), nb


def conv2d_fwd(x, wp, bias, cop, R, S, stride, pad, pad_mode="zero", act="none", slope=0.0,
               out=None, role="fwd", co_real=None):
    """co_real: the real output channels when cop pads them (vst_conv2d_fwd_co)."""
    _dev_check(x, wp, bias)
    if co_real is not None and co_real < cop:
        N, H, W, Cx = x.shape
        Ho = (H + 2 * pad - R) // stride + 1
        Wo = (W + 2 * pad - S) // stride + 1
        y = out if out is not None else torch.empty((N, Ho, Wo, cop), device=x.device)
        nb = int(lib().vst_conv2d_fwd_co_ws_bytes(N, H, W, Cx, cop, R, S, stride, pad, PAD[pad_mode], int(co_real)))
        ws = torch.empty((nb + 3) // 4, device=x.device) if nb else None
        _call("vst_conv2d_fwd_co_ws", _p(x), _p(wp), _p(getattr(wp, "vst_split", None)), _p(bias), _p(y), N, H, W,
              Cx, cop, R, S, stride, pad, PAD[pad_mode], ACT[act], float(slope), _math(role), int(co_real), _p(ws), nb,
              _stream())
        return y
    N, H, W, Cx = x.shape
    Ho = (H + 2 * pad - R) // stride + 1
    Wo = (W + 2 * pad - S) // stride + 1
    y = out if out is not None else torch.empty((N, Ho, Wo, cop), device=x.device)
    m = _math(role)
    ws, nb = _fwd_ws(N, H, W, Cx, cop, R, S, stride, pad, m, x.device) if S == R else (None, 0)
    h = _probe_begin("fwd", (N, H, W, Cx, cop, R, stride, pad, pad_mode)) if _probes else None
    if ws is not None:
        _call("vst_conv2d_fwd_ws", _p(x), _p(wp), _p(getattr(wp, "vst_split", None)), _p(bias), _p(y), N, H, W, Cx,
              cop, R, S, stride, pad, PAD[pad_mode], ACT[act], float(slope), m, None, None, _p(ws), nb, _stream())
    else:
        _call("vst_conv2d_fwd", _p(x), _p(wp), _p(getattr(wp, "vst_split", None)), _p(bias), _p(y), N, H,
              W, Cx, cop, R, S, stride, pad,
              PAD[pad_mode], ACT[act], float(slope), m, _stream())
    _probe_end(h)
    return y


def conv2d_fwd_in(x, wp, bias, cop, R, S, stride, pad, pad_mode="zero", role="fwd"):
    """A conv that feeds an InstanceNorm: (y, stats).  The split-bf16 kernels emit the statistics
    partials from their epilogue (vst_conv2d_fwd_in) and one small fold finalizes them; other paths
    (fp32 policy, 4-channel inputs, image sizes not a multiple of 32 pixels) fall back to
    instnorm_stats(y).  Same stats layout as instnorm_stats."""
    import ctypes
    _dev_check(x, wp, bias)
    N, H, W, Cx = x.shape
    Ho = (H + 2 * pad - R) // stride + 1
    Wo = (W + 2 * pad - S) // stride + 1
    y = torch.empty((N, Ho, Wo, cop), device=x.device)
    hw = Ho * Wo
    part = torch.empty((N * max(1, hw // 32) * cop * 2,), device=x.device, dtype=torch.float64)
    nsplit = ctypes.c_int(0)
    m = _math(role)
    ws, nb = _fwd_ws(N, H, W, Cx, cop, R, S, stride, pad, m, x.device) if S == R else (None, 0)
    h = _probe_begin("fwd", (N, H, W, Cx, cop, R, stride, pad, pad_mode)) if _probes else None
    _call("vst_conv2d_fwd_ws", _p(x), _p(wp), _p(getattr(wp, "vst_split", None)), _p(bias), _p(y), N, H, W, Cx,
          cop, R, S, stride, pad, PAD[pad_mode], ACT["none"], 0.0, m, _p(part),
          ctypes.addressof(nsplit), _p(ws), nb, _stream())
    _probe_end(h)
    if nsplit.value == 0:
        return y, instnorm_stats(y)
    stats = torch.empty((N, cop, 2), device=x.device)
    _call("vst_instnorm_finalize", _p(part), _p(stats), N, hw, cop, nsplit.value, IN_EPS, _stream())
    return y, stats


def conv2d_tfwd(x, wp, bias, Ho, Wo, cx, R, S, stride, pad, act="none", slope=0.0,
                pad_mode="zero", addend=None, role="bwd", co_real=None):
    """Transposed conv / data gradient (vst_conv2d_tfwd).  pad_mode='reflect' (stride 1) is the
    exact gradient of ReflectionPad2d(pad)+conv; addend is added in the epilogue.  co_real: the real
    channels of x when Cy pads them (vst_conv2d_tfwd_co: the PatchGAN head's data gradient)."""
    _dev_check(x, wp, bias, addend)
    N, Hi, Wi, Cy = x.shape
    y = torch.empty((N, Ho, Wo, cx), device=x.device)
    if co_real is not None and co_real < Cy:
        _call("vst_conv2d_tfwd_co", _p(x), _p(wp), _p(bias), _p(addend), _p(y), N, Hi, Wi, Cy, Ho, Wo, cx,
              R, S, stride, pad, PAD[pad_mode], ACT[act], float(slope), _math(role), int(co_real), _stream())
        return y
    _call("vst_conv2d_tfwd", _p(x), _p(wp), _p(bias), _p(addend), _p(y), N, Hi, Wi, Cy, Ho, Wo, cx,
          R, S, stride, pad, PAD[pad_mode], ACT[act], float(slope), _math(role), _stream())
    return y


# The weight gradient over the NHWC operands (vst_conv2d_wgrad_nhwc: x fp32 NHWC, dy as its NHWC bf16 planes) where
# the shape takes it; False: the channel-major operand images of vst_conv2d_wgrad_pre.
WGRAD_NHWC = True
# ... and with dy fp32 NHWC itself (vst_conv2d_wgrad_nhwc_f32: the stride-2 convs, the ConvTranspose and
# PatchGAN weight gradients, whose dy has no planes): no operand image at all.
WGRAD_NHWC_F32 = True
# ... and its im2col form for output rows shorter than 32 pixels (vst_conv2d_wgrad_nhwc_f32: the StarGAN discriminator's
# 16x16 / 8x8 / 4x4 layers)
WGRAD_IM2COL = True


@functools.lru_cache(maxsize=512)
def _wgrad_nhwc_plan_ok(N, H, W, Cx, Ho, Wo, Cyp, R, stride, pad, math):
    return bool(lib().vst_conv2d_wgrad_nhwc_ok(N, H, W, Cx, Ho, Wo, Cyp, R, R, stride, pad, math))


def wgrad_nhwc_ok(N, H, W, Cx, Ho, Wo, Cyp, R, stride, pad, policy=None, role="bwd"):
    """Does vst_conv2d_wgrad_nhwc take this shape under the current policy (policy: accepted for the callers' cache
    keys; the arithmetic is the current policy's)?"""
    return WGRAD_NHWC and _wgrad_nhwc_plan_ok(N, H, W, Cx, Ho, Wo, Cyp, R, stride, pad, _math(role))


@functools.lru_cache(maxsize=512)
def _wgrad_nhwc_f32_plan_ok(N, H, W, Cx, Ho, Wo, Cyp, R, stride, pad, math):
    return bool(lib().vst_conv2d_wgrad_nhwc_f32_ok(N, H, W, Cx, Ho, Wo, Cyp, R, R, stride, pad, math))


def wgrad_nhwc_f32_ok(N, H, W, Cx, Ho, Wo, Cyp, R, stride, pad, role="bwd"):
    """... the fp32-dy form (vst_conv2d_wgrad_nhwc_f32, including its im2col form for short output rows): then no
    operand image need be made for this weight gradient (the producers of x and dy write NHWC fp32 only)."""
    if not WGRAD_NHWC_F32:
        return False
    m = _math(role)
    return (_wgrad_nhwc_plan_ok(N, H, W, Cx, Ho, Wo, Cyp, R, stride, pad, m) or
            (WGRAD_IM2COL and _wgrad_nhwc_f32_plan_ok(N, H, W, Cx, Ho, Wo, Cyp, R, stride, pad, m)))


def conv2d_wgrad(x, dy, dw, db, R, S, stride, pad, pad_mode, co, ci, so, si, accumulate=True,
                 role="bwd", dy_planes=None, x_t=None, dy_apl=None):
    """dw (+)= weight gradient written with strides (so, si) — see vst_conv2d_wgrad; db (if not
    None) (+)= per-channel sum of dy (the bias gradient).  dy_planes: dy's bf16 plane image made by
    instnorm_act_bwd(..., planes=True), x_t: x's padded channel-major image made by
    instnorm_act_fwd(..., cp=...) (vst_conv2d_wgrad_pre; both used on the x6 split-bf16 path).
    dy_apl: dy's NHWC bf16 planes (``dy.vst_apl``, instnorm_act_bwd(apre=True)): with x itself (no x_t) the
    NHWC-operand kernel (vst_conv2d_wgrad_nhwc) where the shape takes it."""
    _dev_check(x, dy)
    N, H, W, Cx = x.shape
    _, Ho, Wo, Cyp = dy.shape
    if dy_apl is None and getattr(dy, "vst_planes_only", False) and dy_planes is None:
        dy_apl = getattr(dy, "vst_apl", None)
    if (dy_apl is not None and x_t is None and S == R and
            wgrad_nhwc_ok(N, H, W, Cx, Ho, Wo, Cyp, R, stride, pad, _policy_name, role)):
        nbytes = int(lib().vst_conv2d_wgrad_nhwc_ws_bytes(N, H, W, Cx, Ho, Wo, Cyp, R, S, stride, pad, _math(role)))
        ws = torch.empty((nbytes + 3) // 4, device=x.device)
        h = _probe_begin("wgrad", (N, H, W, Cx, Cyp, R, stride, pad, pad_mode)) if _probes else None
        _call("vst_conv2d_wgrad_nhwc", _p(x), _p(dy_apl), _p(dw), _p(ws), nbytes, N, H, W, Cx, Ho, Wo, Cyp, R, S, stride,
              pad, PAD[pad_mode], co, ci, so, si, 1 if accumulate else 0, _math(role), _stream())
        _probe_end(h)
        if db is not None:
            if getattr(dy, "vst_planes_only", False):
                raise RuntimeError("conv2d_wgrad: the bias gradient of a planes-only dy comes from its IN backward")
            channel_sum(dy, db, co, accumulate)
        return
    if getattr(dy, "vst_planes_only", False) and dy_planes is None:
        raise RuntimeError("conv2d_wgrad: dy has NHWC planes only and this shape needs its fp32 image / plane copy")
    if (dy_apl is None and x_t is None and dy_planes is None and S == R and
            wgrad_nhwc_f32_ok(N, H, W, Cx, Ho, Wo, Cyp, R, stride, pad, role)):
        nbytes = int(lib().vst_conv2d_wgrad_nhwc_f32_ws_bytes(N, H, W, Cx, Ho, Wo, Cyp, R, S, stride, pad, _math(role)))
        ws = torch.empty((nbytes + 3) // 4, device=x.device)
        h = _probe_begin("wgrad", (N, H, W, Cx, Cyp, R, stride, pad, pad_mode)) if _probes else None
        _call("vst_conv2d_wgrad_nhwc_f32", _p(x), _p(dy), _p(dw), _p(ws), nbytes, N, H, W, Cx, Ho, Wo, Cyp, R, S, stride,
              pad, PAD[pad_mode], co, ci, so, si, 1 if accumulate else 0, _math(role), _stream())
        _probe_end(h)
        if db is not None:
            channel_sum(dy, db, co, accumulate)
        return
    nbytes = lib().vst_conv2d_wgrad_ws_bytes(N, H, W, Cx, Ho, Wo, Cyp, R, S, stride)
    ws = torch.empty((nbytes + 3) // 4, device=x.device)
    h = _probe_begin("wgrad", (N, H, W, Cx, Cyp, R, stride, pad, pad_mode)) if _probes else None
    if db is not None and dy_planes is None and x_t is None:
        # the weight and bias gradient in one fused pass where a route takes the shape (vst_conv2d_wgrad_bias)
        rc = lib().vst_conv2d_wgrad_bias(_p(x), _p(dy), _p(dw), _p(db), _p(ws), nbytes, N, H, W, Cx, Ho, Wo, Cyp, R, S,
                                         stride, pad, PAD[pad_mode], co, ci, so, si, 1 if accumulate else 0,
                                         _math(role), _stream())
        if rc == 0:
            _probe_end(h)
            return
        if rc != EUNSUPPORTED:
            _lib.check(rc, "vst_conv2d_wgrad_bias")
    _call("vst_conv2d_wgrad_pre", _p(x), _p(x_t), _p(dy), _p(dy_planes), _p(dw), _p(ws), nbytes, N, H, W, Cx, Ho, Wo,
          Cyp, R, S, stride, pad, PAD[pad_mode], co, ci, so, si, 1 if accumulate else 0, _math(role),
          _stream())
    _probe_end(h)
    if db is not None:
        channel_sum(dy, db, co, accumulate)


# Conv GEMM arithmetic by role (see VST_MATH_* in include/vst_hip.h).  The default policy, bf16x6,
# runs EVERY conv — training forwards, data gradients, weight gradients, inference — with the
# fp32-equivalent three-plane bf16 split (dropped product terms <= 2^-24 relative).  "mixed" (the
# round-1 default) keeps the forwards at bf16x6 — the forward rounding decides ReLU masks, and a mask
# flipped by a 1e-5 perturbation changes which gradients exist (measured on the reference-golden G:
# bf16x3 forward => 6e-3 input-grad error, bf16x6 forward => 1e-7) — but runs data/weight gradients
# and inference-only forwards at bf16x3 (~2^-16 relative products, ~1e-5 relative gradient error):
# narrower than fp32, so it is a separately labelled option.  VST_CONV_MATH / set_conv_math:
# bf16x6 (default) | mixed | fp32 (v_mfma_f32_32x32x2_f32) | bf16x3.
_POLICIES = {"mixed": {"fwd": "bf16x6", "infer": "bf16x3", "bwd": "bf16x3"},
             "fp32": {"fwd": "fp32", "infer": "fp32", "bwd": "fp32"},
             "bf16x3": {"fwd": "bf16x3", "infer": "bf16x3", "bwd": "bf16x3"},
             "bf16x6": {"fwd": "bf16x6", "infer": "bf16x6", "bwd": "bf16x6"}}
_policy_name = os.environ.get("VST_CONV_MATH", "bf16x6")
if _policy_name not in _POLICIES:
    raise ValueError("VST_CONV_MATH must be one of %s" % sorted(_POLICIES))


def set_conv_math(policy):
    """Select the conv arithmetic policy (fp32 | bf16x3 | bf16x6 | mixed); returns the previous."""
    global _policy_name
    if policy not in _POLICIES:
        raise ValueError(policy)
    prev, _policy_name = _policy_name, policy
    return prev


def get_conv_math():
    return _policy_name


# Deterministic debug switch: the warp input gradients (warp_bwd_nhwc,
# warp_masked_bwd_nhwc, the temporal loss's ga) run the atomic-free sort + ordered-gather path
# (vst_warp_bwd_input_det) instead of the fp32-atomic scatter, so two runs agree bit for bit.
_deterministic = os.environ.get("VST_DETERMINISTIC", "0") == "1"


def set_deterministic(flag):
    """Select the deterministic warp backward (True) or the atomic scatter (False); returns the previous."""
    global _deterministic
    prev, _deterministic = _deterministic, bool(flag)
    return prev


def _warp_bwd_det(gout, flow, gx, align_corners, masked, negate, cl):
    N, H, W, C = gout.shape
    ws = torch.empty(lib().vst_warp_bwd_det_ws_bytes(N, H, W), device=gout.device, dtype=torch.uint8)
    _call("vst_warp_bwd_input_det", _p(gout), _p(flow), _p(gx), _p(ws), ws.numel(), N, H, W, C, cl,
          int(align_corners), int(masked), int(negate), _stream())


def _math(role):
    from ._lib import MATH_MODES
    return MATH_MODES[_POLICIES[_policy_name][role]]


def debug_set_tiles(fprop=-1, tconv=-1, wgrad=-1):
    """Force GEMM tiles for calls from this host thread (vst_debug_set_tiles; -1 = automatic).  The cached
    route answers depend on the planner's tiles: dropped."""
    lib().vst_debug_set_tiles(int(fprop), int(tconv), int(wgrad))
    _wgrad_nhwc_plan_ok.cache_clear()
    _wgrad_nhwc_f32_plan_ok.cache_clear()


PLAN_RK, PLAN_SKINNY, PLAN_C4_DIRECT = -1, -2, -3
TILE_NAMES = {0: "128x128 (8 waves of 64x32)", 1: "128x64", 2: "128x128 (4 waves of 64x64)", 3: "64x128",
              4: "128x128 BK64", 5: "128x64 BK64", 6: "64x64", 7: "256x128 (8 waves of 64x64)", 8: "64x64 BK64",
              9: "128x128 BK16 (4 waves of 64x64, 2 blocks/CU at x6)",
              PLAN_RK: "fp32 [row][k] kernel", PLAN_SKINNY: "VALU skinny kernel",
              PLAN_C4_DIRECT: "4-channel patch-staged direct kernel"}


WPLAN_NAMES = {0: "conv_wgrad_k (NHWC operands)", 1: "copies + conv_wgrad_rk_k", 2: "copies + conv_wgrad_bf_k",
               3: "skinny VALU", 4: "Wo-padded copies + conv_wgrad_bf_k"}


def conv_plan_wgrad(N, H, W, Cx, Ho, Wo, Cyp, R, S, stride, math):
    """Host-only query (vst_conv_plan_wgrad): (path, tile kind, nsplit) of vst_conv2d_wgrad."""
    import ctypes
    from ._lib import MATH_MODES
    m = MATH_MODES[math] if math in MATH_MODES else _math(math)
    path, kind, ns = ctypes.c_int(0), ctypes.c_int(0), ctypes.c_int(0)
    _call("vst_conv_plan_wgrad", N, H, W, Cx, Ho, Wo, Cyp, R, S, stride, m, ctypes.addressof(path),
          ctypes.addressof(kind), ctypes.addressof(ns))
    return path.value, kind.value, ns.value


def conv_plan_fwd_tail(N, H, W, Cx, Cop, R, S, stride, pad, math):
    """Host-only: split-K count of the x6 tail launch vst_conv2d_fwd_ws runs for this shape (0: none)."""
    import ctypes
    from ._lib import MATH_MODES
    m = MATH_MODES[math] if math in MATH_MODES else _math(math)
    ks = ctypes.c_int(0)
    _call("vst_conv_plan_fwd_tail", N, H, W, Cx, Cop, R, S, stride, pad, m, ctypes.addressof(ks))
    return ks.value


def conv_plan_fwd(N, H, W, Cx, Cop, R, S, stride, pad_h, pad_w, math, with_tail=False):
    """Host-only query (vst_conv_plan_fwd): (tile kind, tail-split row[, tail kind]) vst_conv2d_fwd
    would use for this shape under `math` ('fp32' | 'bf16x3' | 'bf16x6', or a role of the current
    policy)."""
    import ctypes
    from ._lib import MATH_MODES
    m = MATH_MODES[math] if math in MATH_MODES else _math(math)
    kind, ms, tk = ctypes.c_int(0), ctypes.c_int(0), ctypes.c_int(0)
    _call("vst_conv_plan_fwd", N, H, W, Cx, Cop, R, S, stride, pad_h, pad_w, m, ctypes.addressof(kind),
          ctypes.addressof(ms), ctypes.addressof(tk))
    return (kind.value, ms.value, tk.value) if with_tail else (kind.value, ms.value)


def channel_sum(x, db, cl, accumulate=True):
    """db[c] (+)= sum over pixels of x[..., c] (bias gradient)."""
    _dev_check(x)
    cs = x.shape[-1]
    nhw = x.numel() // cs
    nbytes = lib().vst_channel_sum_ws_bytes(nhw, cs)
    ws = torch.empty((nbytes + 3) // 4, device=x.device)
    _call("vst_channel_sum", _p(x), _p(db), _p(ws), nhw, cs, cl, 1 if accumulate else 0, _stream())


# ReflectionPad2d(1) + 3x3 data gradients as the interior conv + border GEMM (vst_conv2d_dgrad_refl)
# instead of the conv over the zero-padded frame + reflect fold; False keeps the fold.
DGRAD_BORDER = True


def conv2d_dgrad_s1(dy, ikf, H, W, cx, R, pad, pad_mode="zero", addend=None, role="bwd"):
    """Data gradient of a stride-1 conv as a FORWARD conv (the split-bf16 MFMA fprop kernel with
    pre-split weights).  Reflect padding, 3x3 / pad 1: the interior dx = conv(dy, rot180(W)^T, zero
    pad 1) (+ addend in its epilogue) plus the padded border positions' GEMM added into rows / columns
    1 and H-2 / W-2 (vst_conv2d_dgrad_refl).  Other reflect cases: dx_full = conv(dy, rot180(W)^T,
    zero pad R-1) over the padded input frame [H+2p][W+2p], then the reflect fold (+ addend).  Zero
    padding p <= R-1: dx = conv(dy, rot180(W)^T, zero pad R-1-p) directly (+ addend).  ikf:
    VST_PACK_IKF pack."""
    _dev_check(dy, ikf, addend)
    if pad_mode == "reflect" and DGRAD_BORDER and R == 3 and pad == 1 and getattr(ikf, "vst_split", None) is not None:
        N, Hy, Wy, Cy = dy.shape
        m = _math(role)
        nb = int(lib().vst_conv2d_dgrad_refl_ws_bytes(N, H, W, Cy, cx, m)) if (Hy, Wy) == (H, W) else 0
        if nb:
            dx = torch.empty((N, H, W, cx), device=dy.device)
            ws = torch.empty((nb + 3) // 4, device=dy.device)
            h = _probe_begin("dgrad", (N, H, W, Cy, cx, R, 1, pad, pad_mode)) if _probes else None
            _call("vst_conv2d_dgrad_refl", _p(dy), _p(ikf.vst_split), _p(addend), _p(dx), _p(ws), nb, N, H, W, Cy, cx,
                  m, _stream())
            _probe_end(h)
            return dx
    if pad_mode == "reflect":
        dxp = conv2d_fwd(dy, ikf, None, cx, R, R, 1, R - 1, "zero", role=role)
        return reflect_fold(dxp, pad, addend)
    if pad > R - 1:
        raise NotImplementedError("conv2d_dgrad_s1: zero padding must be <= R-1")
    dx = conv2d_fwd(dy, ikf, None, cx, R, R, 1, R - 1 - pad, "zero", role=role)
    if addend is not None:
        axpby(addend, dx, 1.0, 1.0)
    return dx


# The data gradient of ReflectionPad2d(p) + Conv2d(C -> 4, 7x7) (the generator's last layer) as the
# zero-pad-p conv of dy on the direct 4-channel kernel + the reflect-fold frame (vst_c4_dgrad_frame),
# instead of the conv over the (H+2p) x (W+2p) padded frame + reflect_fold.  False: that route.
C4_DGRAD = True


def c4_dgrad_reflect_ok(dy, cx, R, pad, role="bwd"):
    N, H, W, C = dy.shape
    return (C4_DGRAD and C == 4 and cx % 16 == 0 and R == 2 * pad + 1 and H > 2 * pad + 1 and W > 2 * pad + 1
            and conv_plan_fwd(N, H, W, 4, cx, R, R, 1, pad, pad, role)[0] == PLAN_C4_DIRECT)


def c4_dgrad_reflect(dy, ikf, H, W, cx, R, pad, role="bwd"):
    """dx of ReflectionPad2d(pad) + Conv2d(cx -> 4, R x R) from the 4-channel dy (ikf: VST_PACK_IKF):
    the interior dxp[i+pad][j+pad] as the zero-pad-pad forward conv over dy (the direct 4-channel
    kernel), then vst_c4_dgrad_frame adds the reflect-fold terms of the padded frame's border."""
    _dev_check(dy, ikf)
    N = dy.shape[0]
    dx = conv2d_fwd(dy, ikf, None, cx, R, R, 1, pad, "zero", role=role)
    _call("vst_c4_dgrad_frame", _p(dy), _p(ikf), _p(dx), N, H, W, cx, R, pad, _stream())
    return dx


def conv2d_dgrad_refl_in(dy, ikf, H, W, cx, y_in, stats, act="relu", slope=0.0, addend=None, db=None,
                         accumulate_db=True, planes=False, role="bwd", apre=False):
    """ReflectionPad2d(1) + 3x3 data gradient (conv2d_dgrad_s1's interior conv + border GEMM) fused with
    the InstanceNorm(+act) backward of the layer below it: returns (g, dy_in[, dy_in_planes]) — g = the
    data gradient (+ addend), dy_in = instnorm_act_bwd(g, y_in, stats, act) — or None when the fused route
    does not support the shape / arithmetic.  The IN partials are taken by the data gradient's GEMM
    epilogue and border add (vst_conv2d_dgrad_refl_epi_part: no partial pass; x6 arithmetic, H W % 32 ==
    0); dy's pre-split planes (``dy.vst_apl``) are its A operand when present, and apre
    writes dy_in as planes only."""
    _dev_check(dy, ikf, addend, y_in, stats)
    if not DGRAD_BORDER or getattr(ikf, "vst_split", None) is None:
        return None
    N, Hy, Wy, Cy = dy.shape
    C = y_in.shape[-1]
    if (Hy, Wy) != (H, W) or cx != C:
        return None
    m = _math(role)
    nb = int(lib().vst_conv2d_dgrad_refl_in_epi_ws_bytes(N, H, W, Cy, C, m))
    if not nb:
        return None
    g = torch.empty((N, H, W, C), device=dy.device)
    dyi = torch.empty_like(g)
    ws = torch.empty((nb + 3) // 4, device=dy.device)
    pl, ldp = None, 0
    if planes:
        ldp = lib().vst_cp_ld(N * H * W)
        pl = torch.empty((3, C, ldp), device=dy.device, dtype=torch.bfloat16)
    if apre:  # dy_in as NHWC planes only (instnorm_act_bwd(apre=True))
        dyi.vst_apl = torch.empty((3, dyi.numel()), device=dy.device, dtype=torch.bfloat16)
        dyi.vst_planes_only = True
    h = _probe_begin("dgrad", (N, H, W, Cy, C, 3, 1, 1, "reflect")) if _probes else None
    _call("vst_conv2d_dgrad_refl_epi_part", _p(dy), _p(getattr(dy, "vst_apl", None)), _p(ikf.vst_split),
          _p(addend), _p(g), _p(y_in), _p(stats), _p(ws), nb, N, H, W, Cy, C, ACT[act], float(slope), m, _stream())
    _probe_end(h)
    _call("vst_instnorm_act_bwd_epi_tail", _p(g), _p(y_in), _p(stats), _p(dyi), _p(db), _p(ws), N, H, W, C, ACT[act],
          float(slope), 1 if accumulate_db else 0, _p(pl), ldp, _p(getattr(dyi, "vst_apl", None)), _stream())
    return (g, dyi, pl) if planes else (g, dyi)


def dgrad_refl_epi_ok(N, H, W, Cy, Cx, role="bwd"):
    """Does conv2d_dgrad_refl_in take this shape (vst_conv2d_dgrad_refl_in_epi_ws_bytes > 0)?"""
    return DGRAD_BORDER and int(lib().vst_conv2d_dgrad_refl_in_epi_ws_bytes(N, H, W, Cy, Cx, _math(role))) > 0


def reflect_fold(dxp, p, addend=None):
    _dev_check(dxp, addend)
    N, Hp, Wp, C = dxp.shape
    H, W = Hp - 2 * p, Wp - 2 * p
    dx = torch.empty((N, H, W, C), device=dxp.device)
    _call("vst_reflect_fold", _p(dxp), _p(addend), _p(dx), N, H, W, C, p, _stream())
    return dx


# --------------------------------------------------------------------------------- instnorm
def _in_ws(N, HW, C, device):
    nbytes = lib().vst_instnorm_ws_bytes(N, HW, C)
    return torch.empty((nbytes + 7) // 8, dtype=torch.float64, device=device)


def instnorm_stats(y):
    _dev_check(y)
    N, H, W, C = y.shape
    stats = torch.empty((N, C, 2), device=y.device)
    ws = _in_ws(N, H * W, C, y.device)
    _call("vst_instnorm_stats", _p(y), _p(stats), _p(ws), N, H * W, C, IN_EPS, _stream())
    return stats


def instnorm_act_fwd(y, stats, act="relu", slope=0.0, residual=None, cp=None, xpl=None):
    """a = act(IN(y)) (+ residual).  cp = (pad, pad_mode, stride) of the conv that consumes a:
    returns (a, a_t) where a_t is a's padded channel-major image for that conv's x6 weight gradient
    (vst_instnorm_act_fwd_cp; conv2d_wgrad(x_t=a_t)).  xpl = (pad, pad_mode, wx): returns (a, planes),
    a's padded image as the bf16 planes [3][C][ld] with wx zero columns per row
    (vst_instnorm_act_fwd_planes; tap_conv_wgrad_swap(x_pl=planes))."""
    _dev_check(y, stats, residual)
    N, H, W, C = y.shape
    a = torch.empty_like(y)
    if xpl is not None:
        pad, mode, wx = xpl
        ld = lib().vst_cp_ld(N * (H + 2 * pad) * (W + 2 * pad + wx))
        pl = torch.empty((3, C, ld), device=y.device, dtype=torch.bfloat16)
        _call("vst_instnorm_act_fwd_planes", _p(y), _p(stats), _p(residual), _p(a), _p(pl), N, H, W, C, ACT[act],
              float(slope), pad, PAD[mode], wx, _stream())
        return a, pl
    if cp is not None:
        pad, mode, st = cp
        at = torch.empty((C, lib().vst_cp_ld(N * (H + 2 * pad) * (W + 2 * pad))), device=y.device)
        _call("vst_instnorm_act_fwd_cp", _p(y), _p(stats), _p(residual), _p(a), _p(at), N, H, W, C, ACT[act],
              float(slope), pad, PAD[mode], st, _stream())
        return a, at
    _call("vst_instnorm_act_fwd", _p(y), _p(stats), _p(residual), _p(a), N, H * W, C, ACT[act],
          float(slope), _stream())
    return a


def instnorm_act_bwd(ga, y, stats, act="relu", slope=0.0, db=None, accumulate_db=True, planes=False, apre=False):
    """dy = backward of act(IN(y)); db (if given) (+)= sum of dy per channel (conv-bias grad).
    planes=True: returns (dy, dy_planes) — the apply pass also writes dy's three bf16 planes
    [3][C][vst_cp_ld(N*H*W)], the x6 weight gradient's operand image (conv2d_wgrad(dy_planes=...)).
    apre: dy is written ONLY as its NHWC bf16 planes ``dy.vst_apl`` (the pre-split A operand of the data
    gradient that consumes it, conv2d_dgrad_refl_in) — dy's fp32 values are NOT written (dy.vst_planes_only):
    its readers must take the planes (the weight gradient: dy_planes; the data gradient: vst_apl)."""
    _dev_check(ga, y, stats)
    N, H, W, C = y.shape
    dy = torch.empty_like(y)
    ws = _in_ws(N, H * W, C, y.device)
    pl, ldp = None, 0
    if planes:
        ldp = lib().vst_cp_ld(N * H * W)
        pl = torch.empty((3, C, ldp), device=y.device, dtype=torch.bfloat16)
    if apre:
        dy.vst_apl = torch.empty((3, dy.numel()), device=y.device, dtype=torch.bfloat16)
        dy.vst_planes_only = True
        _call("vst_instnorm_act_bwd_planes_apre", _p(ga), _p(y), _p(stats), _p(dy), _p(db), _p(ws), N, H * W, C,
              ACT[act], float(slope), 1 if accumulate_db else 0, _p(pl), ldp, _p(dy.vst_apl), _stream())
        return (dy, pl) if planes else dy
    _call("vst_instnorm_act_bwd_planes", _p(ga), _p(y), _p(stats), _p(dy), _p(db), _p(ws), N, H * W, C,
          ACT[act], float(slope), 1 if accumulate_db else 0, _p(pl), ldp, _stream())
    return (dy, pl) if planes else dy


def act_bwd(gy, y, act, slope=0.0):
    _dev_check(gy, y)
    dx = torch.empty_like(y)
    _call("vst_act_bwd", _p(gy), _p(y), _p(dx), y.numel(), ACT[act], float(slope), _stream())
    return dx


# ------------------------------------------------------------------------------------- flow
def warp_nhwc(x, flow, align_corners=False):
    _dev_check(x, flow)
    N, H, W, C = x.shape
    out = torch.empty_like(x)
    _call("vst_warp_fwd", _p(x), _p(flow), _p(out), N, H, W, C, int(align_corners), _stream())
    return out


def warp_bwd_nhwc(gout, flow, align_corners=False):
    _dev_check(gout, flow)
    N, H, W, C = gout.shape
    gx = torch.zeros_like(gout)
    if _deterministic:
        _warp_bwd_det(gout, flow, gx, align_corners, False, False, C)
        return gx
    _call("vst_warp_bwd_input", _p(gout), _p(flow), _p(gx), N, H, W, C, int(align_corners), _stream())
    return gx


def fbcheck(ff, bf):
    _dev_check(ff, bf)
    N, _, H, W = bf.shape
    mask = torch.empty((N, 1, H, W), device=bf.device)
    _call("vst_fbcheck", _p(ff), _p(bf), _p(mask), N, H, W, _stream())
    return mask


# ----------------------------------------------------------------------------------- losses
def _part(npix, device):
    return torch.empty(lib().vst_loss_part_floats(npix), device=device)


def loss_temporal(a, b, flow, mask, lam, cl=3):
    _dev_check(a, b, flow, mask)
    N, H, W, Cs = a.shape
    loss = torch.empty((), device=a.device)
    _call("vst_loss_temporal", _p(a), _p(b), _p(flow), _p(mask), _p(loss), _p(_part(N * H * W, a.device)),
          N, H, W, Cs, cl, float(lam), _stream())
    return loss


def loss_temporal_bwd(a, b, flow, mask, gout, ga, gb, lam, cl=3):
    N, H, W, Cs = a.shape
    if _deterministic and ga is not None:   # gb first, then ga -= its ordered scatter
        gbuf = gb if gb is not None else torch.empty_like(a)
        _call("vst_loss_temporal_bwd", _p(a), _p(b), _p(flow), _p(mask), _p(gout), None, _p(gbuf), N, H, W,
              Cs, cl, float(lam), _stream())
        _warp_bwd_det(gbuf, flow, ga, False, False, True, cl)
        return
    _call("vst_loss_temporal_bwd", _p(a), _p(b), _p(flow), _p(mask), _p(gout), _p(ga), _p(gb), N, H, W,
          Cs, cl, float(lam), _stream())


def loss_l1(a, b, scale, cl=3):
    _dev_check(a, b)
    npix = a.numel() // a.shape[-1]
    loss = torch.empty((), device=a.device)
    _call("vst_loss_l1", _p(a), _p(b), _p(loss), _p(_part(npix, a.device)), npix, a.shape[-1], cl,
          float(scale), _stream())
    return loss


def loss_l1_bwd(a, b, gout, scale, cl=3):
    npix = a.numel() // a.shape[-1]
    g = torch.empty_like(a)
    _call("vst_loss_l1_bwd", _p(a), _p(b), _p(gout), _p(g), npix, a.shape[-1], cl, float(scale), _stream())
    return g


def loss_mse_const(a, target, scale=1.0, cl=1):
    _dev_check(a)
    npix = a.numel() // a.shape[-1]
    loss = torch.empty((), device=a.device)
    _call("vst_loss_mse_const", _p(a), float(target), _p(loss), _p(_part(npix, a.device)), npix,
          a.shape[-1], cl, float(scale), _stream())
    return loss


def loss_mse_const_bwd(a, target, gout, scale=1.0, cl=1):
    npix = a.numel() // a.shape[-1]
    g = torch.empty_like(a)
    _call("vst_loss_mse_const_bwd", _p(a), float(target), _p(gout), _p(g), npix, a.shape[-1], cl,
          float(scale), _stream())
    return g


# -------------------------------------------------------------------------------- optimizer
def adam_step(p, g, m, v, lr, beta1, beta2, eps, step):
    _dev_check(p, g, m, v)
    _call("vst_adam_step", _p(p), _p(g), _p(m), _p(v), p.numel(), float(lr), float(beta1),
          float(beta2), float(eps), int(step), _stream())


def axpby(x, y, a, b):
    _dev_check(x, y)
    _call("vst_axpby", _p(x), _p(y), x.numel(), float(a), float(b), _stream())


# ------------------------------------------------------------- learning-based style path
def warp_masked_nhwc(x, flow, align_corners=False):
    """fs_lib.warp (methods/learning-based/fs_lib.py:5-39): warp * grid_sample(ones) validity."""
    _dev_check(x, flow)
    N, H, W, C = x.shape
    out = torch.empty_like(x)
    _call("vst_warp_masked_fwd", _p(x), _p(flow), _p(out), N, H, W, C, int(align_corners), _stream())
    return out


def warp_masked_bwd_nhwc(gout, flow, align_corners=False):
    _dev_check(gout, flow)
    N, H, W, C = gout.shape
    gx = torch.zeros_like(gout)
    if _deterministic:
        _warp_bwd_det(gout, flow, gx, align_corners, True, False, C)
        return gx
    _call("vst_warp_masked_bwd_input", _p(gout), _p(flow), _p(gx), N, H, W, C, int(align_corners),
          _stream())
    return gx


def instnorm_affine_fwd(y, stats, gamma, beta, act="none", gate=None, gate_mult=1.0, residual=None,
                        slope=0.0):
    """s * act(gamma * IN(y) + beta) + residual (vst_instnorm_affine_fwd); gamma/beta padded to C."""
    _dev_check(y, stats, gamma, beta, gate, residual)
    N, H, W, C = y.shape
    out = torch.empty_like(y)
    _call("vst_instnorm_affine_fwd", _p(y), _p(stats), _p(gamma), _p(beta), _p(gate), float(gate_mult),
          _p(residual), _p(out), N, H * W, C, ACT[act], float(slope), _stream())
    return out


def instnorm_affine_bwd(g, y, stats, gamma, beta, act="none", gate=None, gate_mult=1.0, dgamma=None,
                        dbeta=None, dgate=None, dbias=None, accumulate=True, slope=0.0):
    _dev_check(g, y, stats, gamma, beta, gate)
    N, H, W, C = y.shape
    dx = torch.empty_like(y)
    nbytes = lib().vst_instnorm_affine_ws_bytes(N, H * W, C)
    ws = torch.empty((nbytes + 7) // 8, dtype=torch.float64, device=y.device)
    _call("vst_instnorm_affine_bwd", _p(g), _p(y), _p(stats), _p(gamma), _p(beta), _p(gate),
          float(gate_mult), _p(dx), _p(dgamma), _p(dbeta), _p(dgate), _p(dbias), _p(ws), N, H * W, C,
          ACT[act], float(slope), 1 if accumulate else 0, _stream())
    return dx


def upsample2x(x):
    _dev_check(x)
    N, H, W, C = x.shape
    y = torch.empty((N, 2 * H, 2 * W, C), device=x.device)
    _call("vst_upsample2x_fwd", _p(x), _p(y), N, H, W, C, _stream())
    return y


def upsample2x_bwd(gy):
    _dev_check(gy)
    N, H2, W2, C = gy.shape
    gx = torch.empty((N, H2 // 2, W2 // 2, C), device=gy.device)
    _call("vst_upsample2x_bwd", _p(gy), _p(gx), N, H2 // 2, W2 // 2, C, _stream())
    return gx


def scaled_tanh(x, cl=3):
    _dev_check(x)
    y = torch.empty_like(x)
    _call("vst_scaled_tanh_fwd", _p(x), _p(y), x.numel() // x.shape[-1], x.shape[-1], cl, _stream())
    return y


def scaled_tanh_bwd(x, gy, cl=3):
    _dev_check(x, gy)
    gx = torch.empty_like(x)
    _call("vst_scaled_tanh_bwd", _p(x), _p(gy), _p(gx), x.numel() // x.shape[-1], x.shape[-1], cl,
          _stream())
    return gx


def channel_normalize(x, mean, std, d0=1.0, cl=3, backward=False):
    """((x / d0) - mean[c]) / std[c] (backward: (x / std[c]) / d0); mean/std device tensors [cl]."""
    _dev_check(x, mean, std)
    y = torch.empty_like(x)
    _call("vst_channel_normalize", _p(x), _p(y), _p(mean), _p(std), float(d0),
          x.numel() // x.shape[-1], x.shape[-1], cl, 1 if backward else 0, _stream())
    return y


def maxpool2(x):
    _dev_check(x)
    N, H, W, C = x.shape
    y = torch.empty((N, H // 2, W // 2, C), device=x.device)
    _call("vst_maxpool2_fwd", _p(x), _p(y), N, H, W, C, _stream())
    return y


def maxpool2_bwd(gy, x):
    _dev_check(gy, x)
    N, H, W, C = x.shape
    gx = torch.empty_like(x)
    _call("vst_maxpool2_bwd", _p(gy), _p(x), _p(gx), N, H, W, C, _stream())
    return gx


def loss_mse(a, b, scale=1.0, cl=None, out=None, accumulate=False):
    """scale * mean((a - b)^2) over the cl logical channels (default all)."""
    _dev_check(a, b)
    cs = a.shape[-1]
    npix = a.numel() // cs
    loss = out if out is not None else torch.zeros((), device=a.device)
    _call("vst_loss_mse", _p(a), _p(b), _p(loss), _p(_part(npix, a.device)), npix, cs, cl or cs,
          float(scale), 1 if accumulate else 0, _stream())
    return loss


def loss_mse_bwd(a, b, gout, scale=1.0, cl=None, grad=None):
    cs = a.shape[-1]
    npix = a.numel() // cs
    acc = grad is not None
    g = grad if acc else torch.empty_like(a)
    _call("vst_loss_mse_bwd", _p(a), _p(b), _p(gout), _p(g), npix, cs, cl or cs, float(scale),
          1 if acc else 0, _stream())
    return g


def loss_tv(img, scale=1.0, cl=3):
    _dev_check(img)
    N, H, W, C = img.shape
    loss = torch.zeros((), device=img.device)
    _call("vst_loss_tv", _p(img), _p(loss), _p(_part(N * (H - 1) * (W - 1), img.device)), N, H, W, C, cl,
          float(scale), 0, _stream())
    return loss


def loss_tv_bwd(img, gout, scale=1.0, cl=3):
    N, H, W, C = img.shape
    g = torch.empty_like(img)
    _call("vst_loss_tv_bwd", _p(img), _p(gout), _p(g), N, H, W, C, cl, float(scale), _stream())
    return g


def gram(f, role="fwd"):
    """G[b] = F_b^T F_b / (h*w) for NHWC features f [B][h][w][C] -> [B][C][C]
    (fast_style_transfer.py:813-817).  Each G[b] is the weight gradient of a 1x1 conv whose input
    and output gradient are both F_b, i.e. the split-K MFMA wgrad kernel."""
    _dev_check(f)
    B, h, w, C = f.shape
    G = torch.empty((B, C, C), device=f.device)
    for b in range(B):
        fb = f[b:b + 1]
        conv2d_wgrad(fb, fb, G[b], None, 1, 1, 1, 0, "zero", C, C, C, 1, accumulate=False, role=role)
    axpby(G, G, 1.0 / (h * w), 0.0)
    return G


def split_planes(wp):
    """Attach the bf16 split planes (vst_weight_split) the split-arithmetic conv paths read."""
    split = torch.empty((3,) + tuple(wp.shape), device=wp.device, dtype=torch.bfloat16)
    _call("vst_weight_split", _p(wp), _p(split), wp.numel(), _stream())
    wp.vst_split = split
    return wp


def gram_bwd(f, dG, role="bwd"):
    """dF_b = F_b (dG_b + dG_b^T) / (h*w): a 1x1 conv of F_b with weight S_b (vst_gram_sym)."""
    _dev_check(f, dG)
    B, h, w, C = f.shape
    df = torch.empty_like(f)
    for b in range(B):
        S = torch.empty((C, 1, 1, C), device=f.device)
        _call("vst_gram_sym", _p(dG[b]), _p(S), C, float(1.0 / (h * w)), _stream())
        split_planes(S)
        conv2d_fwd(f[b:b + 1], S, None, C, 1, 1, 1, 0, out=df[b:b + 1], role=role)
    return df


def corr_pyramid_floats(P, H2, W2, ld0, levels):
    return lib().vst_corr_pyramid_floats(P, H2, W2, ld0, levels)


def corr_pyramid(pyr, P, H2, W2, ld0, levels):
    _call("vst_corr_pyramid", _p(pyr), P, H2, W2, ld0, levels, _stream())


def corr_lookup(pyr, coords, B, H1, W1, H2, W2, ld0, levels, radius, cs=None):
    """cs: the output channel stride (default cpad; the padded channels are written as zeros)."""
    _dev_check(pyr, coords)
    K = 2 * radius + 1
    cs = cs or cpad(levels * K * K)
    out = torch.empty((B, H1, W1, cs), device=pyr.device)
    _call("vst_corr_lookup", _p(pyr), _p(coords), _p(out), B, H1, W1, H2, W2, ld0, levels, radius, cs,
          _stream())
    return out


# -------------------------------------------------------------------------------- StarGAN
def concat_label_nhwc(x, label, cs=None):
    """NCHW x [N,Cx,H,W] + label [N,Cl] -> NHWC [N,H,W,cs] (StarGAN model.py:59-64)."""
    _dev_check(x, label)
    N, Cx, H, W = x.shape
    Cl = label.shape[1]
    cs = cs or cpad(Cx + Cl)
    y = torch.empty((N, H, W, cs), device=x.device)
    _call("vst_concat_label_nhwc", _p(x), _p(label), _p(y), N, Cx, Cl, H, W, cs, _stream())
    return y


def instnorm_running_update(stats, running_mean, running_var, HW, momentum=0.1):
    _dev_check(stats, running_mean, running_var)
    N, C, _ = stats.shape
    _call("vst_instnorm_running_update", _p(stats), _p(running_mean), _p(running_var), N, C, HW,
          float(momentum), IN_EPS, _stream())


def instnorm_stats_from_running(running_mean, running_var, N):
    _dev_check(running_mean, running_var)
    C = running_mean.numel()
    stats = torch.empty((N, C, 2), device=running_mean.device)
    _call("vst_instnorm_stats_from_running", _p(running_mean), _p(running_var), _p(stats), N, C, IN_EPS,
          _stream())
    return stats


# -------------------------------------------------------------------------------- formats
def fc2_unpack(raw):
    """raw float32 [B,H,W,9] FC2 block on the device -> (img1 NHWC4, img2 NHWC4, mask [B,1,H,W],
    flow [B,2,H,W]) as the CycleGANCon step consumes them (fc2_dataset.py:35-41)."""
    _dev_check(raw)
    B, H, W, nine = raw.shape
    if nine != 9 or raw.dtype != torch.float32 or not raw.is_contiguous():
        raise ValueError("fc2_unpack: expected contiguous float32 [B,H,W,9]")
    img1 = torch.empty((B, H, W, 4), device=raw.device)
    img2 = torch.empty((B, H, W, 4), device=raw.device)
    mask = torch.empty((B, 1, H, W), device=raw.device)
    flow = torch.empty((B, 2, H, W), device=raw.device)
    _call("vst_fc2_unpack", _p(raw), _p(img1), _p(img2), _p(mask), _p(flow), B, H, W, _stream())
    return img1, img2, mask, flow


def u8_image_to_nhwc4(x):
    """uint8 [B,H,W,3] on the device -> ToTensor + Normalize(0.5, 0.5) as float32 NHWC4."""
    if not x.is_cuda:
        raise RuntimeError("vst ops require GPU tensors (no CPU fallback)")
    if x.dtype != torch.uint8 or x.shape[-1] != 3 or not x.is_contiguous():
        raise ValueError("u8_image_to_nhwc4: expected contiguous uint8 [..., 3]")
    y = torch.empty(tuple(x.shape[:-1]) + (4,), device=x.device)
    _call("vst_u8_image_to_nhwc4", _p(x), _p(y), x.numel() // 3, _stream())
    return y


# ----------------------------------------------------------------------------------- RAFT
# conv2d_fwd_hw with the split-K plans of the square convs' workspace path (RAFT's SepConvGRU convs);
# False: the one-launch plans
FWD_HW_SPLITK = True


def conv2d_fwd_hw(x, wp, bias, cop, R, S, stride, pad_h, pad_w, act="none", role="fwd"):
    """Forward conv with separate row / column zero padding (vst_conv2d_fwd_hw)."""
    _dev_check(x, wp, bias)
    N, H, W, Cx = x.shape
    Ho = (H + 2 * pad_h - R) // stride + 1
    Wo = (W + 2 * pad_w - S) // stride + 1
    y = torch.empty((N, Ho, Wo, cop), device=x.device)
    m = _math(role)
    nb = int(lib().vst_conv2d_fwd_hw_ws_bytes(N, H, W, Cx, cop, R, S, stride, pad_h, pad_w, m)) if FWD_HW_SPLITK else 0
    if nb:  # the split-K plans for small grids (vst_conv2d_fwd_hw_ws)
        ws = torch.empty((nb + 3) // 4, device=x.device)
        _call("vst_conv2d_fwd_hw_ws", _p(x), _p(wp), _p(getattr(wp, "vst_split", None)), _p(bias), _p(y), N, H, W,
              Cx, cop, R, S, stride, pad_h, pad_w, ACT[act], 0.0, m, _p(ws), nb, _stream())
        return y
    _call("vst_conv2d_fwd_hw", _p(x), _p(wp), _p(getattr(wp, "vst_split", None)), _p(bias), _p(y), N, H, W, Cx,
          cop, R, S, stride, pad_h, pad_w, ACT[act], 0.0, m, _stream())
    return y


def raft_prep(img, pads, nhwc=False, out=None):
    """[B,3,H,W] NCHW (or NHWC [B,H,W,Cs>=3] with nhwc=True) -> replicate pad (l, r, t, b) +
    2*(x/255)-1 -> NHWC4 (written into ``out`` when given)."""
    _dev_check(img, out)
    l, r, t, b = pads
    if nhwc:
        B, H, W, cs = img.shape
    else:
        B, C, H, W = img.shape
        if C != 3:
            raise ValueError("raft_prep: expected 3-channel images")
    shape = (B, H + t + b, W + l + r, 4)
    if out is None:
        out = torch.empty(shape, device=img.device)
    elif tuple(out.shape) != shape:
        raise ValueError("raft_prep: out has shape %s, expected %s" % (tuple(out.shape), shape))
    if nhwc:
        _call("vst_raft_prep_nhwc", _p(img), cs, _p(out), B, H, W, l, r, t, b, _stream())
        return out
    _call("vst_raft_prep", _p(img), _p(out), B, H, W, l, r, t, b, _stream())
    return out


def add_relu(a, b, out=None):
    _dev_check(a, b, out)
    y = out if out is not None else torch.empty_like(a)
    _call("vst_add_relu", _p(a), _p(b), _p(y), a.numel(), _stream())
    return y


def copy_channels(src, src_c0, dst, dst_c0, nc):
    _dev_check(src, dst)
    npix = src.numel() // src.shape[-1]
    if dst.numel() // dst.shape[-1] != npix:
        raise ValueError("copy_channels: pixel counts differ")
    _call("vst_copy_channels", _p(src), src.shape[-1], src_c0, _p(dst), dst.shape[-1], dst_c0, nc, npix, _stream())


def raft_ctx_split(c, hdim, cdim, h, hx, rhx):
    _dev_check(c, h, hx, rhx)
    npix = c.numel() // c.shape[-1]
    _call("vst_raft_ctx_split", _p(c), c.shape[-1], hdim, cdim, _p(h), _p(hx), _p(rhx), hx.shape[-1], npix,
          _stream())


def raft_flow4(coords1, flow4):
    _dev_check(coords1, flow4)
    B, _, h, w = coords1.shape
    _call("vst_raft_flow4", _p(coords1), _p(flow4), B, h, w, _stream())


def raft_motion(out, nout, flow4, hx, rhx, c0):
    _dev_check(out, flow4, hx, rhx)
    npix = out.numel() // out.shape[-1]
    _call("vst_raft_motion", _p(out), out.shape[-1], nout, _p(flow4), _p(hx), _p(rhx), hx.shape[-1], c0, npix,
          _stream())


def gru_reset(zr, h, rhx):
    _dev_check(zr, h, rhx)
    hd = h.shape[-1]
    _call("vst_gru_reset", _p(zr), _p(h), _p(rhx), hd, rhx.shape[-1], h.numel() // hd, _stream())


def gru_update(zr, q, h, hx):
    _dev_check(zr, q, h, hx)
    hd = h.shape[-1]
    _call("vst_gru_update", _p(zr), _p(q), _p(h), _p(hx), hd, hx.shape[-1], h.numel() // hd, _stream())


def raft_coords_update(coords1, delta):
    _dev_check(coords1, delta)
    B, _, h, w = coords1.shape
    _call("vst_raft_coords_update", _p(coords1), _p(delta), delta.shape[-1], B, h, w, _stream())


def raft_upsample(coords1, mask):
    _dev_check(coords1, mask)
    B, _, h, w = coords1.shape
    out = torch.empty((B, 2, 8 * h, 8 * w), device=coords1.device)
    _call("vst_raft_upsample", _p(coords1), _p(mask), mask.shape[-1], _p(out), B, h, w, _stream())
    return out


def loss_masked_l1(a, b, mask, scale, cl):
    """scale * mean(mask * |a - b|) over cl logical channels of NHWC a, b; mask [B,1,H,W] / [B,H,W] or None."""
    _dev_check(a, b, mask)
    npix = a.numel() // a.shape[-1]
    loss = torch.empty((), device=a.device)
    _call("vst_loss_masked_l1", _p(a), _p(b), _p(mask), _p(loss), _p(_part(npix, a.device)), npix, a.shape[-1], cl,
          float(scale), _stream())
    return loss


def loss_masked_l1_bwd(a, b, mask, gout, scale, cl):
    _dev_check(a, b, mask, gout)
    npix = a.numel() // a.shape[-1]
    grad = torch.empty_like(a)
    _call("vst_loss_masked_l1_bwd", _p(a), _p(b), _p(mask), _p(gout), _p(grad), npix, a.shape[-1], cl, float(scale),
          _stream())
    return grad


# ----------------------------------------------------------------------- tap-GEMM convolutions
# VST_TAP_CHUNK_MB > 0 runs the tap GEMMs' R*R*4-wide intermediates (411 MB for 8 images at 256^2,
# 7x7) in chunks of images sized for the 256 MB Infinity Cache, each chunk overwriting one buffer.
# Off by default: the C2 step A/B measured 63.15-63.27 ms with 128 MB chunks, 64.12 with 64 MB,
# 62.85-62.87 in one pass (the smaller GEMM launches lose more than the cache hits save).
TAP_CHUNK_BYTES = 0
# tap_conv_wgrad: the folded dy written as the x6 wgrad's bf16 planes (vst_tapfold_planes);
# False writes the fp32 D and lets the wgrad copy it into planes.
TAP_PLANES = True
# The generator's last-layer weight gradient as the swapped GEMM (tap_conv_wgrad_swap); False:
# the R x 1 form (tap_conv_wgrad_h).
TAP_SWAP = True


def _tap_chunks(N, per_image_bytes):
    n = N if TAP_CHUNK_BYTES <= 0 else max(1, min(N, TAP_CHUNK_BYTES // max(1, per_image_bytes)))
    return [(i, min(N, i + n)) for i in range(0, N, n)]


def tap_conv_fwd(x, ck, bias, R, pad, pad_mode="zero", act="none", slope=0.0, role="fwd"):
    """'same' conv with <= 4 output channels on the MFMA kernel (see vst_tapsum_fwd): ck is the
    VST_PACK_CK pack [R][S][4][Ci] of the weight, bias padded to 4 (or None); returns NHWC4."""
    _dev_check(x, ck, bias)
    N, H, W, Cx = x.shape
    if ck.shape != (R, R, 4, Cx):
        raise ValueError("tap_conv_fwd: CK pack shape %s does not match R=%d, Cx=%d" % (tuple(ck.shape), R, Cx))
    y = torch.empty((N, H, W, 4), device=x.device)
    chunks = _tap_chunks(N, H * W * R * R * 16)
    zbuf = torch.empty((chunks[0][1], H, W, R * R * 4), device=x.device)
    for a, b in chunks:
        z = conv2d_fwd(x[a:b], ck, None, R * R * 4, 1, 1, 1, 0, "zero", role=role, out=zbuf[:b - a])
        _call("vst_tapsum_fwd", _p(z), R * R * 4, _p(bias), _p(y[a:b]), b - a, H, W, R, R, pad, PAD[pad_mode],
              ACT[act], float(slope), _stream())
    return y


def tap_conv_fwd_h(x, sok, bias, R, pad, pad_mode="zero", act="none", slope=0.0, role="fwd"):
    """The same conv as tap_conv_fwd with the (r, ci) contraction on the matrix cores and only the column
    taps summed afterwards (vst_tapconv_h_fwd): sok = the VST_PACK_SOK pack [S*4][R][1][Ci]."""
    _dev_check(x, sok, bias)
    N, H, W, Cx = x.shape
    if sok.shape != (R * 4, R, 1, Cx):
        raise ValueError("tap_conv_fwd_h: SOK pack shape %s does not match R=%d, Cx=%d" % (tuple(sok.shape), R, Cx))
    Ho, Wo = H + 2 * pad - R + 1, W + 2 * pad - R + 1
    y = torch.empty((N, Ho, Wo, 4), device=x.device)
    z = torch.empty((N, Ho, W, R * 4), device=x.device)
    _call("vst_tapconv_h_fwd", _p(x), _p(sok), _p(getattr(sok, "vst_split", None)), _p(bias), _p(z), _p(y), N, H, W,
          Cx, R, pad, PAD[pad_mode], ACT[act], float(slope), _math(role), _stream())
    return y


def tap_conv_wgrad(x, dy, dw, R, pad, pad_mode="zero", accumulate=True, role="bwd", x_t=None):
    """dw [Co<=4][Ci][R][R] (+)= weight gradient of tap_conv_fwd given dy NHWC4 (pre-activation).
    x_t: x's unpadded channel-major image (instnorm_act_fwd(cp=(0, "zero", 1))) for the x6 path."""
    _dev_check(x, dy, dw)
    N, H, W, Cx = x.shape
    Co, Ci = dw.shape[0], dw.shape[1]
    K = R * R * 4
    if TAP_PLANES and TAP_CHUNK_BYTES <= 0 and conv_plan_wgrad(N, H, W, Cx, H, W, K, 1, 1, 1, role)[0] == 2:
        # D straight as the x6 wgrad's bf16 planes (vst_tapfold_planes): no fp32 D, no plane copy
        P = N * H * W
        ldp = lib().vst_cp_ld(P)
        pl = torch.empty((3, K, ldp), device=x.device, dtype=torch.bfloat16)
        _call("vst_tapfold_planes", _p(dy), _p(pl), ldp, N, H, W, R, R, pad, PAD[pad_mode], _stream())
        t = torch.empty((K, Ci), device=x.device)
        nbytes = lib().vst_conv2d_wgrad_ws_bytes(N, H, W, Cx, H, W, K, 1, 1, 1)
        ws = torch.empty((nbytes + 3) // 4, device=x.device)
        _call("vst_conv2d_wgrad_pre", _p(x), _p(x_t), _p(pl), _p(pl), _p(t), _p(ws), nbytes, N, H, W, Cx, H, W, K, 1, 1, 1,
              0, PAD["zero"], K, Ci, Ci, 1, 0, _math(role), _stream())
        _call("vst_tap_wgrad_scatter", _p(t), _p(dw), Co, Ci, R, R, 1 if accumulate else 0, _stream())
        return
    chunks = _tap_chunks(N, H * W * R * R * 16)
    dbuf = torch.empty((chunks[0][1], H, W, R * R * 4), device=x.device)
    t = torch.empty((R * R * 4, Ci), device=x.device)
    for a, b in chunks:
        d = dbuf[:b - a]
        _call("vst_tapfold", _p(dy[a:b]), _p(d), b - a, H, W, R, R, pad, PAD[pad_mode], _stream())
        conv2d_wgrad(x[a:b], d, t, None, 1, 1, 1, 0, "zero", R * R * 4, Ci, Ci, 1, accumulate=a > 0, role=role)
    _call("vst_tap_wgrad_scatter", _p(t), _p(dw), Co, Ci, R, R, 1 if accumulate else 0, _stream())


def tap_conv_wgrad_h_ok(x, R, pad, pad_mode, role="bwd"):
    """Does tap_conv_wgrad_h take this shape: a reflect 'same' conv whose R x 1 wgrad frame (W+R+1 wide)
    runs on the x6 split-bf16 kernel without padded rows."""
    N, H, W, Cx = x.shape
    return (pad_mode == "reflect" and 2 * pad == R - 1 and pad + 1 < min(H, W) and
            conv_plan_wgrad(N, H, W, Cx, H + 2, W + R + 1, 4 * R, R, 1, 1, role)[0] == 2)


def tap_conv_wgrad_h(x, dy, dw, R, pad, pad_mode="reflect", accumulate=True, role="bwd", x_t=None):
    """tap_conv_wgrad as the R x 1 conv's weight gradient (vst_tapshift_planes): dy's column-shifted copies
    as 4R channels over the (H+2) x (W+R+1) frame, x padded by pad+1.  x_t: x's channel-major image padded
    by pad+1, reflect (instnorm_act_fwd(cp=(pad + 1, "reflect", 1))), or None."""
    _dev_check(x, dy, dw)
    N, H, W, Cx = x.shape
    Co, Ci = dw.shape[0], dw.shape[1]
    K = 4 * R
    Ho, Wo = H + 2, W + R + 1
    ldp = lib().vst_cp_ld(N * Ho * Wo)
    pl = torch.empty((3, K, ldp), device=x.device, dtype=torch.bfloat16)
    _call("vst_tapshift_planes", _p(dy), _p(pl), ldp, N, H, W, R, _stream())
    t = torch.empty((K, Ci, R), device=x.device)
    nbytes = lib().vst_conv2d_wgrad_ws_bytes(N, H, W, Cx, Ho, Wo, K, R, 1, 1)
    ws = torch.empty((nbytes + 3) // 4, device=x.device)
    _call("vst_conv2d_wgrad_pre", _p(x), _p(x_t), _p(pl), _p(pl), _p(t), _p(ws), nbytes, N, H, W, Cx, Ho, Wo, K, R, 1,
          1, pad + 1, PAD["reflect"], K, Ci, Ci * R, R, 0, _math(role), _stream())
    _call("vst_tap_wgrad_scatter_h", _p(t), _p(dw), Co, Ci, R, R, 1 if accumulate else 0, _stream())


def tap_swap_geom(W, R):
    """(wx, frame width) of tap_conv_wgrad_swap: the (W+R-1)-wide reflect-padded x rows get wx zero
    columns so that every row is whole 8-pixel chunks."""
    wx = (8 - (W + R - 1) % 8) % 8
    return wx, W + R - 1 + wx


def tap_conv_wgrad_swap_ok(x, R, pad, pad_mode, role="bwd", co=4):
    """Does tap_conv_wgrad_swap take this shape: a reflect 'same' conv whose swapped GEMM (the R x R wgrad
    of the dy channels against x's padded frame as Ci outputs) runs on the x6 split-bf16 kernel.  co: the
    layer's real output channels — vst_tap_wgrad_swap runs the GEMM over 3 dy channels when co <= 3, 4
    otherwise, and the plan is queried with that same count."""
    N, H, W, Cx = x.shape
    wx, Wq = tap_swap_geom(W, R)
    cx = 3 if co <= 3 else 4
    return (TAP_SWAP and pad_mode == "reflect" and 2 * pad == R - 1 and pad < min(H, W) and Cx % 4 == 0 and
            conv_plan_wgrad(N, H, W + wx, cx, H + R - 1, Wq, Cx, R, R, 1, role)[0] == 2)


def tap_conv_wgrad_swap(x, dy, dw, R, pad, pad_mode="reflect", accumulate=True, role="bwd", x_pl=None, db=None):
    """tap_conv_wgrad with the GEMM's roles swapped (vst_tap_wgrad_swap): M = R*R*3 (tap, co) rows of the
    zero-padded dy against x's reflect-padded frame as Cx columns.  x_pl: that frame's bf16 planes as the
    IN apply writes them (instnorm_act_fwd(xpl=(pad, "reflect", wx))); None: made here from x."""
    _dev_check(x, dy, dw)
    N, H, W, Cx = x.shape
    Co, Ci = dw.shape[0], dw.shape[1]
    if pad_mode != "reflect" or 2 * pad != R - 1:
        raise NotImplementedError("tap_conv_wgrad_swap: reflect 'same' convs only")
    if tuple(dy.shape) != (N, H, W, 4) or Co > 4 or Ci != Cx:
        raise ValueError("tap_conv_wgrad_swap: dy %s / dw %s do not match x %s" % (tuple(dy.shape), tuple(dw.shape),
                                                                               tuple(x.shape)))
    if x_pl is None:  # the identity IN (mean 0, rstd 1): a == x, plus the planes
        st = torch.zeros((N, Cx, 2), device=x.device)
        st[..., 1] = 1.0
        _, x_pl = instnorm_act_fwd(x, st, "none", xpl=(pad, "reflect", tap_swap_geom(W, R)[0]))
    ld = lib().vst_tap_wgrad_swap_ld(N, H, W, R)
    if x_pl.shape != (3, Cx, ld) or x_pl.dtype != torch.bfloat16:
        raise ValueError("tap_conv_wgrad_swap: x planes %s do not match (3, %d, %d) bf16" % (tuple(x_pl.shape), Cx, ld))
    nbytes = lib().vst_tap_wgrad_swap_ws_bytes(N, H, W, Cx, R)
    ws = torch.empty((nbytes + 3) // 4, device=x.device)
    # db: the bias gradient (+)= the channel sums of dy, taken by the same pass (vst_tap_wgrad_swap_db)
    _call("vst_tap_wgrad_swap_db", _p(dy), _p(x_pl), _p(dw), _p(db), _p(ws), nbytes, N, H, W, Cx, R, Co,
          1 if accumulate else 0, _math(role), _stream())


def tap_conv_dgrad(dy, kc, R, pad, pad_mode="zero", role="bwd"):
    """Data gradient (NHWC4) of a 'same' conv with <= 4 input channels: kc = VST_PACK_KC pack
    [R][R][4][Cy] of its weight (see vst_tapgather)."""
    _dev_check(dy, kc)
    N, H, W, Cy = dy.shape
    if kc.shape != (R, R, 4, Cy):
        raise ValueError("tap_conv_dgrad: KC pack shape %s does not match R=%d, Cy=%d" % (tuple(kc.shape), R, Cy))
    y = torch.empty((N, H, W, 4), device=dy.device)
    chunks = _tap_chunks(N, H * W * R * R * 16)
    zbuf = torch.empty((chunks[0][1], H, W, R * R * 4), device=dy.device)
    for a, b in chunks:
        z = conv2d_fwd(dy[a:b], kc, None, R * R * 4, 1, 1, 1, 0, "zero", role=role, out=zbuf[:b - a])
        _call("vst_tapgather", _p(z), _p(y[a:b]), b - a, H, W, R, R, pad, PAD[pad_mode], _stream())
    return y


def dgrad_sok_pack(w, ci_real=None):
    """VST_PACK_SOK pack of the data gradient of a conv with <= 4 input channels, w [Co][Ci][R][S]: the
    conv dy -> dx over the taps rotated 180 deg, w_d[o = ci][i = co][r][s] = w[co][ci][R-1-r][S-1-s].
    ci_real: only the first ci_real (<= 4) input channels' gradient (the others' is not wanted)."""
    Co, Ci, R, S = w.shape
    Ci = ci_real or Ci
    pb = PackBatch._active
    if pb is not None:  # straight from w: transposed strides + reversed tap maps
        return pb.add(w, PACK_SOK, Ci, Co, R, S, (R * S, w.shape[1] * R * S, S, 1), list(range(R - 1, -1, -1)),
                      list(range(S - 1, -1, -1)), Op=4)
    return weight_pack(w.detach()[:, :Ci].permute(1, 0, 2, 3).flip(2, 3).contiguous(), PACK_SOK, Op=4)


def tap_conv_dgrad_h(dy, sokd, R, pad, pad_mode="zero", role="bwd"):
    """Data gradient (NHWC4) of a 'same' conv with <= 4 input channels via vst_tapconv_h_fwd: the full
    correlation of dy with the rotated taps (sokd = dgrad_sok_pack(w); zero pad R-1), then the reflect fold
    (reflect padding) or the interior crop (zero padding)."""
    _dev_check(dy, sokd)
    if pad_mode == "reflect" and pad != (R - 1) // 2:
        raise NotImplementedError("tap_conv_dgrad_h: reflect padding %d with R=%d (only 'same', (R-1)/2)" % (pad, R))
    full = tap_conv_fwd_h(dy, sokd, None, R, R - 1, "zero", role=role)
    if pad_mode == "reflect":
        return reflect_fold(full, pad)
    o = R - 1 - pad
    return full[:, o:full.shape[1] - o, o:full.shape[2] - o].contiguous()


def convT3s2_phase_packs(wt):
    """Phase weight packs of a ConvTranspose2d(k=3, stride=2, padding=1, output_padding=1) weight
    wt [Ci][Co][3][3]: output parity a (rows) / b (cols) uses taps k=1 (even) or k=(2, 0) at input
    offsets (0, +1) (odd).  Returns the VST_PACK_OK packs of the 1x1, 1x2, 2x1, 2x2 phase convs."""
    pb = PackBatch._active
    if pb is not None:  # packed straight from wt (transposed view + tap maps), no copies
        Ci, Co = wt.shape[0], wt.shape[1]
        st = (9, Co * 9, 3, 1)  # logical [o = co][i = ci][a][b] of wt[ci][co][kh][kw]
        return [pb.add(wt, PACK_OK, Co, Ci, 1 + a, 1 + b, st, [2, 0] if a else [1], [2, 0] if b else [1])
                for a, b in ((0, 0), (0, 1), (1, 0), (1, 1))]
    wc = wt.detach().permute(1, 0, 2, 3)  # [Co][Ci][kh][kw]
    odd = torch.tensor([2, 0], device=wt.device)
    ev = torch.tensor([1], device=wt.device)
    packs = []
    for a, b in ((0, 0), (0, 1), (1, 0), (1, 1)):
        w = wc.index_select(2, odd if a else ev).index_select(3, odd if b else ev).contiguous()
        packs.append(weight_pack(w, PACK_OK))
    return packs


def conv4s2_dgrad_phase_packs(w):
    """Phase packs of the data gradient of Conv2d(k=4, stride 2, padding 1) with weight w [Co][Ci][4][4]:
    output parity a (rows) / b (cols) = a 2x2 conv over dy (padding 1) with taps (3, 1) (even) or
    (2, 0) (odd) of w read as [out = ci][in = co] (VST_PACK_OK packs, PackBatch tap maps)."""
    Co, Ci = w.shape[0], w.shape[1]
    maps = ([3, 1], [2, 0])
    pb = PackBatch._active
    if pb is not None:
        st = (16, Ci * 16, 4, 1)  # logical [o = ci][i = co][r][s] of w[co][ci][kh][kw]
        return [pb.add(w, PACK_OK, Ci, Co, 2, 2, st, maps[a], maps[b]) for a, b in ((0, 0), (0, 1), (1, 0), (1, 1))]
    wc = w.detach().permute(1, 0, 2, 3)
    packs = []
    for a, b in ((0, 0), (0, 1), (1, 0), (1, 1)):
        ra, cb = torch.tensor(maps[a], device=w.device), torch.tensor(maps[b], device=w.device)
        packs.append(weight_pack(wc.index_select(2, ra).index_select(3, cb).contiguous(), PACK_OK))
    return packs


# the four phases in one launch stored interleaved (vst_conv4s2_dgrad); False: images + interleave
C4S2_GROUPED = True


def conv4s2_dgrad(dy, packs, cop, role="bwd"):
    """Data gradient of Conv2d(k=4, s=2, p=1) onto a (2*Hd) x (2*Wd) input via four 2x2 phase convs
    (padding 1, outputs (Hd+1) x (Wd+1)) + vst_interleave_phases_full."""
    _dev_check(dy)
    N, Hd, Wd, Cy = dy.shape
    m = _math(role)
    # a grid of fewer than half a CU round of 128x128 phase tiles (the StarGAN discriminator's deep layers: 100
    # rows x 1024 channels per phase at B = 4, K = 8192) runs as four split-K forwards + the interleave instead
    small = 4 * (-(-N * (Hd + 1) * (Wd + 1) // 128)) * (-(-cop // 128)) < 128
    if C4S2_GROUPED and m != _lib.MATH_MODES["fp32"] and Cy % 32 == 0 and cop != 4 and not small and \
            all(getattr(wp, "vst_split", None) is not None for wp in packs):
        # one launch, stored straight into the interleaved gradient (vst_conv4s2_dgrad)
        y = torch.empty((N, 2 * Hd, 2 * Wd, cop), device=dy.device)
        _call("vst_conv4s2_dgrad", _p(dy), *[_p(wp.vst_split) for wp in packs], _p(y), N, Hd, Wd, Cy, cop, m,
              _stream())
        return y
    outs = [conv2d_fwd(dy, wp, None, cop, 2, 2, 1, 1, "zero", role=role) for wp in packs]
    y = torch.empty((N, 2 * Hd, 2 * Wd, cop), device=dy.device)
    _call("vst_interleave_phases_full", _p(outs[0]), _p(outs[1]), _p(outs[2]), _p(outs[3]), _p(y), N, Hd, Wd,
          cop, _stream())
    return y


# ConvTranspose2d phase convs storing straight into the interleaved output (vst_conv2d_fwd_phase)
# instead of four phase images + vst_interleave_phases; False keeps the latter.
CONVT_DIRECT = True
# ... and all four in one launch (vst_conv2d_convT_s2) where Cx % 32 == 0; False: one per phase.
CONVT_GROUPED = True


def convT3s2_fwd(x, packs, bias, cop, act="none", role="fwd"):
    """ConvTranspose2d(k=3, s=2, p=1, op=1) forward on NHWC x via four phase convs, stored straight into
    the interleaved output (split-bf16 math) or as phase images + interleave."""
    _dev_check(x, bias)
    N, H, W, Cx = x.shape
    m = _math(role)
    if CONVT_DIRECT and m != _lib.MATH_MODES["fp32"] and Cx % 8 == 0 and cop != 4 and \
            all(getattr(wp, "vst_split", None) is not None for wp in packs):
        y = torch.empty((N, 2 * H, 2 * W, cop), device=x.device)
        if CONVT_GROUPED and Cx % 32 == 0:
            _call("vst_conv2d_convT_s2", _p(x), *[_p(wp.vst_split) for wp in packs], _p(bias), _p(y), N, H, W, Cx,
                  cop, ACT[act], 0.0, m, _stream())
            return y
        for (a, b), wp in zip(((0, 0), (0, 1), (1, 0), (1, 1)), packs):
            _call("vst_conv2d_fwd_phase", _p(x), _p(wp.vst_split), _p(bias), _p(y), N, H, W, Cx, cop, a, b, ACT[act],
                  0.0, m, _stream())
        return y
    outs = []
    for (a, b), wp in zip(((0, 0), (0, 1), (1, 0), (1, 1)), packs):
        outs.append(conv2d_fwd_hw(x, wp, bias, cop, 1 + a, 1 + b, 1, a, b, act=act, role=role))
    y = torch.empty((N, 2 * H, 2 * W, cop), device=x.device)
    _call("vst_interleave_phases", _p(outs[0]), _p(outs[1]), _p(outs[2]), _p(outs[3]), _p(y), N, H, W, cop,
          _stream())
    return y


_ROUTE_FLAGS = ("FWD_SPLITK", "FWD_HW_SPLITK", "DGRAD_BORDER", "C4_DGRAD", "TAP_CHUNK_BYTES", "TAP_PLANES", "TAP_SWAP",
                "C4S2_GROUPED", "CONVT_DIRECT", "CONVT_GROUPED")
# the forward-route switches of networks.py (the generator's / discriminator's layer routes)
_NET_ROUTE_FLAGS = ("C8_EDGES", "C4_FWD", "DGRAD_AS_FPROP", "TAP_LAST", "TAP_H", "CONVT_PHASES", "IN_XT", "D_CO1")


def route_flags():
    """The module-level route switches that change which kernels a forward launches (tests and tools
    flip them in-process): part of FlatNet.graphed_forward's capture key."""
    import sys
    g = globals()
    net = sys.modules.get(__name__.rsplit(".", 1)[0] + ".networks")
    return tuple(g[n] for n in _ROUTE_FLAGS) + (tuple(getattr(net, n) for n in _NET_ROUTE_FLAGS) if net else ())


_lib.apply_route_overrides(__name__, globals())
