"""TEST INFRASTRUCTURE ONLY (never on the product path): the warp input gradient summed in a FIXED order,
the checker of the deterministic warp backward (csrc/flow_det.hip, vst_warp_bwd_input_det).

The warp is utils/flowtools.py:18-32 (and CycleGANCon/models/cycle_gan_model.py:191-204): F.grid_sample
bilinear with zeros padding, grid = 2 * (pixel + flow) / max(size - 1, 1) - 1.  Its input gradient
scatters w_k(p) * gout[p] to the 4 corners k of every output pixel p.  Here the scatter is a sequential
loop in ascending (p, k) order (k = nw, ne, sw, se) with one fp32 rounding per multiply and per add — the
order the deterministic kernel fixes — so the comparison is bit-exact.  The corner weights follow ATen's
CPU grid sampler arithmetic (the same the product warp is bit-exact to, tests/golden/warp.npz):
ix = fma(g + 1, size / 2, -0.5) (align_corners False) or (g + 1) * ((size - 1) / 2) (True).
Parity of the weights themselves is pinned by the warp golden (the forward shares them).
"""
import numpy as np

f32 = np.float32


def _src_index(g, size, align):
    if align:
        return (g + f32(1)) * f32((size - 1) * 0.5)
    # fma in float64: (g + 1) * (size / 2) is exact there (24-bit x 12-bit), then one rounding to f32
    return ((g + f32(1)).astype(np.float64) * (size * 0.5) - 0.5).astype(f32)


def corner_weights(flow, H, W, align=False):
    """flow [N][2][H][W] f32 -> (x0, y0, [nw, ne, sw, se]) per output pixel, each [N][H][W]."""
    N = flow.shape[0]
    w = np.broadcast_to(np.arange(W, dtype=f32)[None, None, :], (N, H, W))
    h = np.broadcast_to(np.arange(H, dtype=f32)[None, :, None], (N, H, W))
    vx, vy = w + flow[:, 0], h + flow[:, 1]
    gx = f32(2.0) * vx / f32(max(W - 1, 1)) - f32(1.0)
    gy = f32(2.0) * vy / f32(max(H - 1, 1)) - f32(1.0)
    ix, iy = _src_index(gx.astype(f32), W, align), _src_index(gy.astype(f32), H, align)
    fx0, fy0 = np.floor(ix), np.floor(iy)
    we, wn = (ix - fx0).astype(f32), (iy - fy0).astype(f32)
    e, s = (f32(1) - we).astype(f32), (f32(1) - wn).astype(f32)
    wts = [(s * e).astype(f32), (s * we).astype(f32), (wn * e).astype(f32), (wn * we).astype(f32)]
    return fx0.astype(np.int64), fy0.astype(np.int64), wts


def warp_bwd_ordered(gout, flow, align=False, masked=False, cl=None, negate=False):
    """gx (NHWC, like gout) = ordered scatter of gout (NHWC, Cs channels; the first cl scattered)."""
    gout, flow = np.asarray(gout, f32), np.asarray(flow, f32)
    N, H, W, Cs = gout.shape
    cl = Cs if cl is None else cl
    x0, y0, wts = corner_weights(flow, H, W, align)
    cy = [y0, y0, y0 + 1, y0 + 1]
    cx = [x0, x0 + 1, x0, x0 + 1]
    inb = [(cy[k] >= 0) & (cy[k] < H) & (cx[k] >= 0) & (cx[k] < W) for k in range(4)]
    ok = np.ones((N, H, W), bool)
    if masked:  # fs_lib.warp validity (methods/learning-based/fs_lib.py:33-39): in-bounds weights summed in order
        m = np.zeros((N, H, W), f32)
        for k in range(4):
            m = (m + np.where(inb[k], wts[k], f32(0))).astype(f32)
        ok = ~(m < f32(0.9999)) & (m > 0)
    # every contribution as (target, p, k) -> sort -> sequential sums per target
    P = N * H * W
    n_idx = np.broadcast_to(np.arange(N)[:, None, None], (N, H, W))
    tgt, src, wk = [], [], []
    pix = np.arange(P).reshape(N, H, W)
    for k in range(4):
        sel = inb[k] & ok
        tgt.append((n_idx * H * W + cy[k] * W + cx[k])[sel])
        src.append(pix[sel] * 4 + k)
        wk.append(wts[k][sel])
    tgt, src, wk = np.concatenate(tgt), np.concatenate(src), np.concatenate(wk)
    order = np.lexsort((src, tgt))
    tgt, src, wk = tgt[order], src[order], wk[order]
    g = gout.reshape(P, Cs)
    gx = np.zeros((P, Cs), f32)
    contrib = (wk[:, None] * g[src // 4, :cl]).astype(f32)
    if negate:
        contrib = -contrib
    for i in range(len(tgt)):
        t = tgt[i]
        gx[t, :cl] = (gx[t, :cl] + contrib[i]).astype(f32)
    return gx.reshape(N, H, W, Cs)
