"""Algorithmic conv FLOPs of a workload, counted by wrapping the gbvst.ops conv entries (measurement
infrastructure for bench.py's secondary rooflines and tools/layertable.py; not on the product path).

Each function maps an op's arguments to (FLOPs, label): 2 x MACs of the convolution the op computes,
with the reference's real channel counts — a 4-channel image stride counts 3 channels, a one-channel
head padded to 4 counts 1 (co_real) — so a padded lane is waste in the roofline, not work.  Transposed
convs / data gradients count the MACs of the forward conv they differentiate.  Only the outermost op of
a nested call counts (a tap route that calls conv2d_fwd internally is one op).

    with Counter() as c:
        run_one_step()
    c.flops            # total
    c.records          # {(op, label): [flops, calls]}
"""
import functools

from gbvst import ops


def real(c):
    return 3 if c == 4 else c


def _fwd(a, k):
    x, cop, R, S, st, pad = a[0], a[3], a[4], a[5], a[6], a[7]
    N, H, W, C = x.shape
    Ho, Wo = (H + 2 * pad - R) // st + 1, (W + 2 * pad - S) // st + 1
    co = k.get("co_real") or real(cop)
    return 2.0 * N * Ho * Wo * real(C) * co * R * S, "conv%dx%d s%d %d->%d @%dx%d N=%d" % (R, S, st, real(C), co, H, W, N)


def _fwd_hw(a, k):
    x, cop, R, S, st, ph, pw = a[0], a[3], a[4], a[5], a[6], a[7], a[8]
    N, H, W, C = x.shape
    Ho, Wo = (H + 2 * ph - R) // st + 1, (W + 2 * pw - S) // st + 1
    return 2.0 * N * Ho * Wo * real(C) * real(cop) * R * S, "conv%dx%d s%d %d->%d @%dx%d N=%d" % (
        R, S, st, real(C), real(cop), H, W, N)


def _wgrad(a, k):
    x, dy, R, S, st, co, ci = a[0], a[1], a[4], a[5], a[6], a[9], a[10]
    N, Ho, Wo, _ = dy.shape
    return 2.0 * N * Ho * Wo * co * ci * R * S, "wgrad %dx%d s%d %d->%d out %dx%d N=%d" % (R, S, st, ci, co, Ho, Wo, N)


def _dgrad_s1(a, k):
    dy, H, W, cx, R = a[0], a[2], a[3], a[4], a[5]
    N, _, _, C = dy.shape
    C = getattr(dy, "vst_real_c", None) or real(C)  # a 3-channel dy padded to 8 (the tap layers' data gradients)
    return 2.0 * N * H * W * C * real(cx) * R * R, "dgrad%dx%d s1 %d->%d @%dx%d N=%d" % (
        R, R, C, real(cx), H, W, N)


def _dgrad_refl(a, k):
    dy, H, W, cx = a[0], a[2], a[3], a[4]
    N, _, _, C = dy.shape
    return 2.0 * N * H * W * C * real(cx) * 9, "dgrad3x3 s1 %d->%d @%dx%d N=%d" % (C, real(cx), H, W, N)


def _tfwd(a, k):
    dy, Ho, Wo, cx, R, S, st = a[0], a[3], a[4], a[5], a[6], a[7], a[8]
    N, Hi, Wi, Cy = dy.shape
    cy = k.get("co_real") or real(Cy)
    return 2.0 * N * Hi * Wi * cy * real(cx) * R * S, "tdgrad %dx%d s%d %d->%d out %dx%d N=%d" % (
        R, S, st, cy, real(cx), Ho, Wo, N)


def _convT(a, k):
    x, cop = a[0], a[3]
    N, H, W, C = x.shape
    return 2.0 * N * H * W * C * real(cop) * 9, "convT/s2-dgrad 3x3 %d->%d in %dx%d N=%d" % (C, real(cop), H, W, N)


def _c4s2(a, k):
    dy, cop = a[0], a[2]
    N, H, W, C = dy.shape
    return 2.0 * N * H * W * C * real(cop) * 16, "dgrad 4x4 s2 %d->%d in %dx%d N=%d" % (C, real(cop), H, W, N)


def _tap(a, k):
    x, R = a[0], a[3] if len(a) > 3 and isinstance(a[3], int) else a[2]
    N, H, W, C = x.shape
    return 2.0 * N * H * W * C * 3 * R * R, "%dx%d %d<->3 tap route @%dx%d N=%d" % (R, R, C, H, W, N)


def _tap_w(a, k):
    x, dw, R = a[0], a[2], a[3]
    N, H, W, _ = x.shape
    co, ci = dw.shape[0], dw.shape[1]
    return 2.0 * N * H * W * co * ci * R * R, "%dx%d 64<->3 tap route @%dx%d N=%d" % (R, R, H, W, N)


def _tap_d(a, k):
    dy, R = a[0], a[2]
    N, H, W, C = dy.shape
    return 2.0 * N * H * W * C * 3 * R * R, "%dx%d 64<->3 tap route @%dx%d N=%d" % (R, R, H, W, N)


def _c4_dgrad(a, k):
    dy, H, W, cx, R = a[0], a[2], a[3], a[4], a[5]
    N = dy.shape[0]
    return 2.0 * N * H * W * 3 * real(cx) * R * R, "%dx%d 64<->3 tap route @%dx%d N=%d" % (R, R, H, W, N)


def _gram(a, k):
    f = a[0]
    N, H, W, C = f.shape
    return 2.0 * N * C * C * H * W, "gram %d @%dx%d N=%d" % (C, H, W, N)


OPS = {"conv2d_fwd": _fwd, "conv2d_fwd_in": _fwd, "conv2d_fwd_hw": _fwd_hw,
       "conv2d_wgrad": _wgrad, "conv2d_dgrad_s1": _dgrad_s1,
       "conv2d_dgrad_refl_in": _dgrad_refl, "conv2d_tfwd": _tfwd, "convT3s2_fwd": _convT, "conv4s2_dgrad": _c4s2,
       "tap_conv_fwd": _tap, "tap_conv_fwd_h": _tap, "tap_conv_wgrad": _tap_w, "tap_conv_wgrad_h": _tap_w,
       "tap_conv_wgrad_swap": _tap_w, "tap_conv_dgrad": _tap_d, "tap_conv_dgrad_h": _tap_d,
       "c4_dgrad_reflect": _c4_dgrad, "gram": _gram, "gram_bwd": _gram}


class Counter:
    """Counts the algorithmic FLOPs of every conv op called inside the block (outermost calls only).
    on_call(name, label, flops, fn, args, kwargs) -> result may replace the call (tools/layertable.py
    times each op with HIP events that way)."""

    def __init__(self, on_call=None):
        self.flops = 0.0
        self.records = {}
        self._depth = 0
        self._orig = {}
        self._on_call = on_call

    def _wrap(self, name, fn, fl):
        @functools.wraps(fn)
        def w(*a, **k):
            if self._depth:
                return fn(*a, **k)
            f, lab = fl(a, k)
            self._depth += 1
            try:
                out = self._on_call(name, lab, f, fn, a, k) if self._on_call else fn(*a, **k)
            finally:
                self._depth -= 1
            self.flops += f
            r = self.records.setdefault((name, lab), [0.0, 0])
            r[0] += f
            r[1] += 1
            return out
        return w

    def __enter__(self):
        for name, fl in OPS.items():
            fn = getattr(ops, name)
            self._orig[name] = fn
            setattr(ops, name, self._wrap(name, fn, fl))
        return self

    def __exit__(self, *exc):
        for name, fn in self._orig.items():
            setattr(ops, name, fn)
        self._orig = {}
        return False
