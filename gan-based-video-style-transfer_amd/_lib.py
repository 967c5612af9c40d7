"""Loader for libvst_hip.so (the C ABI declared in include/vst_hip.h).

The product path has no fallback: if the shared library is missing or fails to load, importing the
ops raises.  The library is built in-tree (``_build/libvst_hip.so``) by :func:`build` with hipcc for
gfx950; it is loaded AFTER torch so that it binds to the HIP runtime torch already loaded
(both export soname libamdhip64.so.7), which keeps torch's streams valid inside the library.
"""
import ctypes
import glob
import os
import subprocess

import torch  # noqa: F401  (must be loaded first: see module docstring)

PKG = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(PKG)
BUILD = os.path.join(PKG, "_build")
LIB_PATH = os.path.join(BUILD, "libvst_hip.so")
# developer A/B runs only: load an alternative build (tools/build_variant.py) instead
LIB_PATH = os.environ.get("VST_LIB_VARIANT") or LIB_PATH
CSRC = os.path.join(PKG, "csrc")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = "gfx950"

_lib = None


def source_stamp():
    """Short hash of the kernel sources (csrc/* + include/vst_hip.h) plus the VST_* environment knobs
    that change what the kernels do: profiling records carry it, and a record whose stamp differs from
    the running code's is not used for its numbers."""
    import hashlib
    h = hashlib.sha1()
    for f in sorted(glob.glob(os.path.join(CSRC, "*"))) + [os.path.join(REPO, "include", "vst_hip.h")]:
        if f.endswith((".hip", ".h")):
            h.update(os.path.basename(f).encode())
            h.update(open(f, "rb").read())
    knobs = sorted((k, v) for k, v in os.environ.items()
                   if k.startswith("VST_") and k not in ("VST_CONV_MATH", "VST_LIB_VARIANT"))
    h.update(repr(knobs).encode())
    return h.hexdigest()[:12]


MATH_MODES = {"fp32": 0, "bf16x3": 1, "bf16x6": 2}  # VST_MATH_* (include/vst_hip.h)

P = ctypes.c_void_p
I = ctypes.c_int
L = ctypes.c_long
F = ctypes.c_float
D = ctypes.c_double
SZ = ctypes.c_size_t

# name -> (restype, argtypes); mirrors include/vst_hip.h
SIGNATURES = {
    "vst_last_error": (ctypes.c_char_p, []),
    "vst_version": (I, []),
    "vst_build_info": (ctypes.c_char_p, []),
    "vst_nchw_to_nhwc": (I, [P, P, I, I, I, I, I, P]),
    "vst_nhwc_to_nchw": (I, [P, P, I, I, I, I, I, P]),
    "vst_weight_pack": (I, [P, P, I, I, I, I, I, I, I, P]),
    "vst_conv2d_fwd": (I, [P, P, P, P, P, I, I, I, I, I, I, I, I, I, I, I, F, I, P]),
    "vst_weight_split": (I, [P, P, L, P]),
    "vst_weight_pack_batch": (I, [P, I, L, P]),
    "vst_conv2d_fwd_in": (I, [P, P, P, P, P, I, I, I, I, I, I, I, I, I, I, I, F, I, P, P, P]),
    "vst_instnorm_finalize": (I, [P, P, I, I, I, I, F, P]),
    "vst_conv2d_tfwd": (I, [P, P, P, P, P, I, I, I, I, I, I, I, I, I, I, I, I, I, F, I, P]),
    "vst_conv2d_tfwd_co": (I, [P, P, P, P, P, I, I, I, I, I, I, I, I, I, I, I, I, I, F, I, I, P]),
    "vst_conv2d_wgrad_bias": (I, [P, P, P, P, P, SZ, I, I, I, I, I, I, I, I, I, I, I, I, I, I, L, L, I, I, P]),
    "vst_conv2d_wgrad_ws_bytes": (SZ, [I, I, I, I, I, I, I, I, I, I]),
    "vst_conv2d_wgrad": (I, [P, P, P, P, SZ, I, I, I, I, I, I, I, I, I, I, I, I, I, I, L, L, I, I, P]),
    "vst_debug_set_tiles": (None, [I, I, I]),
    "vst_conv_plan_fwd": (I, [I, I, I, I, I, I, I, I, I, I, I, P, P, P]),
    "vst_conv_plan_wgrad": (I, [I, I, I, I, I, I, I, I, I, I, I, P, P, P]),
    "vst_reflect_fold": (I, [P, P, P, I, I, I, I, I, P]),
    "vst_channel_sum_ws_bytes": (SZ, [L, I]),
    "vst_channel_sum": (I, [P, P, P, L, I, I, I, P]),
    "vst_instnorm_ws_bytes": (SZ, [I, I, I]),
    "vst_instnorm_stats": (I, [P, P, P, I, I, I, F, P]),
    "vst_instnorm_act_fwd": (I, [P, P, P, P, I, I, I, I, F, P]),
    "vst_instnorm_act_bwd": (I, [P, P, P, P, P, P, I, I, I, I, F, I, P]),
    "vst_instnorm_act_bwd_planes": (I, [P, P, P, P, P, P, I, I, I, I, F, I, P, L, P]),
    "vst_conv2d_wgrad_nhwc_ok": (I, [I, I, I, I, I, I, I, I, I, I, I, I]),
    "vst_conv2d_wgrad_nhwc_ws_bytes": (SZ, [I, I, I, I, I, I, I, I, I, I, I, I]),
    "vst_conv2d_wgrad_nhwc": (I, [P, P, P, P, SZ, I, I, I, I, I, I, I, I, I, I, I, I, I, I, L, L, I, I, P]),
    "vst_conv2d_wgrad_nhwc_f32_ok": (I, [I, I, I, I, I, I, I, I, I, I, I, I]),
    "vst_conv2d_wgrad_nhwc_f32_ws_bytes": (SZ, [I, I, I, I, I, I, I, I, I, I, I, I]),
    "vst_conv2d_wgrad_nhwc_f32": (I, [P, P, P, P, SZ, I, I, I, I, I, I, I, I, I, I, I, I, I, I, L, L, I, I, P]),
    "vst_conv2d_wgrad_pre": (I, [P, P, P, P, P, P, SZ, I, I, I, I, I, I, I, I, I, I, I, I, I, I, L, L, I, I, P]),
    "vst_instnorm_act_fwd_cp": (I, [P, P, P, P, P, I, I, I, I, I, F, I, I, I, P]),
    "vst_instnorm_act_fwd_planes": (I, [P, P, P, P, P, I, I, I, I, I, F, I, I, I, P]),
    "vst_cp_ld": (L, [L]),
    "vst_conv2d_fwd_co": (I, [P, P, P, P, P, I, I, I, I, I, I, I, I, I, I, I, F, I, I, P]),
    "vst_conv2d_fwd_co_ws_bytes": (SZ, [I, I, I, I, I, I, I, I, I, I, I]),
    "vst_conv2d_fwd_co_ws": (I, [P, P, P, P, P, I, I, I, I, I, I, I, I, I, I, I, F, I, I, P, SZ, P]),
    "vst_tapfold_planes": (I, [P, P, L, I, I, I, I, I, I, I, P]),
    "vst_conv2d_fwd_ws_bytes": (SZ, [I, I, I, I, I, I, I, I, I, I]),
    "vst_conv2d_fwd_ws": (I, [P, P, P, P, P, I, I, I, I, I, I, I, I, I, I, I, F, I, P, P, P, SZ, P]),
    "vst_c4_dgrad_frame": (I, [P, P, P, I, I, I, I, I, I, P]),
    "vst_conv_plan_fwd_tail": (I, [I, I, I, I, I, I, I, I, I, I, P]),
    "vst_act_bwd": (I, [P, P, P, L, I, F, P]),
    "vst_warp_fwd": (I, [P, P, P, I, I, I, I, I, P]),
    "vst_warp_bwd_input": (I, [P, P, P, I, I, I, I, I, P]),
    "vst_fbcheck": (I, [P, P, P, I, I, I, P]),
    "vst_loss_part_floats": (I, [L]),
    "vst_loss_temporal": (I, [P, P, P, P, P, P, I, I, I, I, I, F, P]),
    "vst_loss_temporal_bwd": (I, [P, P, P, P, P, P, P, I, I, I, I, I, F, P]),
    "vst_loss_l1": (I, [P, P, P, P, L, I, I, F, P]),
    "vst_loss_l1_bwd": (I, [P, P, P, P, L, I, I, F, P]),
    "vst_loss_mse_const": (I, [P, F, P, P, L, I, I, F, P]),
    "vst_loss_mse_const_bwd": (I, [P, F, P, P, L, I, I, F, P]),
    "vst_finish_sum": (I, [P, I, P, D, P]),
    "vst_adam_step": (I, [P, P, P, P, L, F, F, F, F, I, P]),
    "vst_axpby": (I, [P, P, L, F, F, P]),
    # learning-based style path / RAFT correlation (style.hip, norm.hip, flow.hip)
    "vst_warp_masked_fwd": (I, [P, P, P, I, I, I, I, I, P]),
    "vst_warp_masked_bwd_input": (I, [P, P, P, I, I, I, I, I, P]),
    "vst_warp_bwd_det_ws_bytes": (SZ, [I, I, I]),
    "vst_warp_bwd_input_det": (I, [P, P, P, P, SZ, I, I, I, I, I, I, I, I, P]),
    "vst_instnorm_affine_fwd": (I, [P, P, P, P, P, F, P, P, I, I, I, I, F, P]),
    "vst_instnorm_affine_ws_bytes": (SZ, [I, I, I]),
    "vst_instnorm_affine_bwd": (I, [P, P, P, P, P, P, F, P, P, P, P, P, P, I, I, I, I, F, I, P]),
    "vst_upsample2x_fwd": (I, [P, P, I, I, I, I, P]),
    "vst_upsample2x_bwd": (I, [P, P, I, I, I, I, P]),
    "vst_scaled_tanh_fwd": (I, [P, P, L, I, I, P]),
    "vst_scaled_tanh_bwd": (I, [P, P, P, L, I, I, P]),
    "vst_channel_normalize": (I, [P, P, P, P, F, L, I, I, I, P]),
    "vst_maxpool2_fwd": (I, [P, P, I, I, I, I, P]),
    "vst_maxpool2_bwd": (I, [P, P, P, I, I, I, I, P]),
    "vst_loss_mse": (I, [P, P, P, P, L, I, I, F, I, P]),
    "vst_loss_mse_bwd": (I, [P, P, P, P, L, I, I, F, I, P]),
    "vst_loss_tv": (I, [P, P, P, I, I, I, I, I, F, I, P]),
    "vst_loss_tv_bwd": (I, [P, P, P, I, I, I, I, I, F, P]),
    "vst_gram_sym": (I, [P, P, I, F, P]),
    "vst_corr_pyramid_floats": (L, [L, I, I, L, I]),
    "vst_corr_pyramid": (I, [P, L, I, I, L, I, P]),
    "vst_corr_lookup": (I, [P, P, P, I, I, I, I, I, L, I, I, I, P]),
    # StarGAN (style.hip, norm.hip)
    "vst_concat_label_nhwc": (I, [P, P, P, I, I, I, I, I, I, P]),
    "vst_instnorm_running_update": (I, [P, P, P, I, I, I, F, F, P]),
    "vst_instnorm_stats_from_running": (I, [P, P, P, I, I, F, P]),
    "vst_fc2_unpack": (I, [P, P, P, P, P, I, I, I, P]),
    "vst_weight_pack_split": (I, [P, P, P, I, I, I, I, I, I, I, P]),
    "vst_conv2d_fwd_hw": (I, [P, P, P, P, P, I, I, I, I, I, I, I, I, I, I, I, F, I, P]),
    "vst_conv2d_fwd_hw_ws_bytes": (SZ, [I, I, I, I, I, I, I, I, I, I, I]),
    "vst_conv2d_fwd_hw_ws": (I, [P, P, P, P, P, I, I, I, I, I, I, I, I, I, I, I, F, I, P, SZ, P]),
    "vst_conv2d_fwd_hwp": (I, [P, P, P, P, P, I, I, I, I, I, I, I, I, I, I, I, I, F, I, P]),
    "vst_tapconv_h_fwd": (I, [P, P, P, P, P, P, I, I, I, I, I, I, I, I, F, I, P]),
    "vst_tapshift_planes": (I, [P, P, L, I, I, I, I, P]),
    "vst_tap_wgrad_scatter_h": (I, [P, P, I, I, I, I, I, P]),
    "vst_conv2d_fwd_phase": (I, [P, P, P, P, I, I, I, I, I, I, I, I, F, I, P]),
    "vst_conv2d_convT_s2": (I, [P, P, P, P, P, P, P, I, I, I, I, I, I, F, I, P]),
    "vst_conv4s2_dgrad": (I, [P, P, P, P, P, P, I, I, I, I, I, I, P]),
    "vst_raft_prep": (I, [P, P, I, I, I, I, I, I, I, P]),
    "vst_tapsum_fwd": (I, [P, I, P, P, I, I, I, I, I, I, I, I, F, P]),
    "vst_tapfold": (I, [P, P, I, I, I, I, I, I, I, P]),
    "vst_tap_wgrad_scatter": (I, [P, P, I, I, I, I, I, P]),
    "vst_tap_wgrad_swap": (I, [P, P, P, P, SZ, I, I, I, I, I, I, I, I, P]),
    "vst_tap_wgrad_swap_db": (I, [P, P, P, P, P, SZ, I, I, I, I, I, I, I, I, P]),
    "vst_tap_wgrad_swap_ws_bytes": (SZ, [I, I, I, I, I]),
    "vst_tap_wgrad_swap_ld": (L, [I, I, I, I]),
    "vst_tapgather": (I, [P, P, I, I, I, I, I, I, I, P]),
    "vst_interleave_phases": (I, [P, P, P, P, P, I, I, I, I, P]),
    "vst_interleave_phases_full": (I, [P, P, P, P, P, I, I, I, I, P]),
    "vst_raft_prep_nhwc": (I, [P, I, P, I, I, I, I, I, I, I, P]),
    "vst_loss_masked_l1": (I, [P, P, P, P, P, L, I, I, F, P]),
    "vst_loss_masked_l1_bwd": (I, [P, P, P, P, P, L, I, I, F, P]),
    "vst_add_relu": (I, [P, P, P, L, P]),
    "vst_copy_channels": (I, [P, I, I, P, I, I, I, L, P]),
    "vst_raft_ctx_split": (I, [P, I, I, I, P, P, P, I, L, P]),
    "vst_raft_flow4": (I, [P, P, I, I, I, P]),
    "vst_raft_motion": (I, [P, I, I, P, P, P, I, I, L, P]),
    "vst_gru_reset": (I, [P, P, P, I, I, L, P]),
    "vst_gru_update": (I, [P, P, P, P, I, I, L, P]),
    "vst_raft_coords_update": (I, [P, P, I, I, I, I, P]),
    "vst_raft_upsample": (I, [P, P, I, P, I, I, I, P]),
    "vst_u8_image_to_nhwc4": (I, [P, P, L, P]),
    "vst_conv2d_dgrad_refl_ws_bytes": (SZ, [I, I, I, I, I, I]),
    "vst_conv2d_dgrad_refl": (I, [P, P, P, P, P, SZ, I, I, I, I, I, I, P]),
    "vst_conv2d_dgrad_refl_in_epi_ws_bytes": (SZ, [I, I, I, I, I, I]),
    "vst_conv2d_dgrad_refl_in_epi": (I, [P, P, P, P, P, P, P, P, P, SZ, I, I, I, I, I, I, F, I, P, L, I, P]),
    "vst_conv2d_dgrad_refl_epi_part": (I, [P, P, P, P, P, P, P, P, SZ, I, I, I, I, I, I, F, I, P]),
    "vst_instnorm_act_bwd_epi_tail": (I, [P, P, P, P, P, P, I, I, I, I, I, F, I, P, L, P, P]),
    "vst_instnorm_act_bwd_planes_apre": (I, [P, P, P, P, P, P, I, I, I, I, F, I, P, L, P, P]),
    # SURVEY §8b spelling (abi.hip)
    "vst_conv_desc_out_hw": (I, [P, P, P]),
    "vst_workspace_size": (SZ, [P, I]),
    "vst_conv2d_fwd_desc": (I, [P, P, P, P, P, P, P, P, P, SZ, P]),
    "vst_conv2d_dgrad_desc": (I, [P, P, P, P, P, P, SZ, P]),
    "vst_conv2d_wgrad_desc": (I, [P, P, P, P, I, I, I, P, SZ, P]),
    "vst_adam_multi_tensor": (I, [P, P, P, P, P, I, F, F, F, F, I, P]),
    "vst_gram_ws_bytes": (SZ, [I, I]),
    "vst_gram": (I, [P, P, I, I, I, P, SZ, I, P]),
    "vst_corr_volume_ws_bytes": (SZ, [I, I, I, I]),
    "vst_corr_volume": (I, [P, P, P, I, I, I, I, I, P, I, P, SZ, I, P]),
    "vst_warp_bilinear_fwd": (I, [P, P, P, I, I, I, I, I, I, P]),
    "vst_warp_bilinear_bwd_input": (I, [P, P, P, I, I, I, I, I, I, P]),
    "vst_masked_sqdiff_mean_fwd": (I, [P, P, P, P, P, P, I, I, I, I, I, F, P]),
    "vst_masked_sqdiff_mean_bwd": (I, [P, P, P, P, P, P, P, I, I, I, I, I, F, P]),
    "vst_l1_mean_fwd": (I, [P, P, P, P, L, I, I, F, P]),
    "vst_l1_mean_bwd": (I, [P, P, P, P, L, I, I, F, P]),
    "vst_mse_const_fwd": (I, [P, F, P, P, L, I, I, F, P]),
    "vst_mse_const_bwd": (I, [P, F, P, P, L, I, I, F, P]),
}


class VstConvDesc(ctypes.Structure):
    """include/vst_hip.h vst_conv_desc."""
    _fields_ = [(n, ctypes.c_int) for n in ("N", "H", "W", "C", "K", "R", "S", "stride", "pad", "pad_mode",
                                             "dilation", "transposed", "output_padding", "layout", "dtype",
                                             "epilogue")] + [("slope", ctypes.c_float), ("math", ctypes.c_int)]


# Per-file compiler flags.  conv_bf.hip: no SLP vectorisation — it pairs the operand split's fp32
# subtractions into v_pk_add_f32, which costs ~22-26 extra cycles each beside MFMAs (MI355X_MICROARCH.md
# cycle constants); scalar v_sub_f32 there: x6 ResnetBlock forward 199 -> 193 us (A/B, same box).
FILE_FLAGS = {"conv_bf.hip": ["-fno-slp-vectorize"]}


def apply_route_overrides(module_name, g):
    """Developer A/B of the mirror's route selectors (module attributes the tests flip in-process): the one
    environment variable VST_ROUTES="ops.WGRAD_NHWC=0,networks.TAP_H=0" sets them at import (tools/ab_step.sh
    arms).  Unknown names raise, so a stale arm cannot silently measure the default."""
    spec = os.environ.get("VST_ROUTES", "").strip()
    if not spec:
        return
    short = module_name.rsplit(".", 1)[-1]
    for item in spec.split(","):
        name, _, val = item.strip().partition("=")
        mod, _, flag = name.partition(".")
        if mod != short:
            continue
        if flag not in g:
            raise ValueError("VST_ROUTES: %s has no route flag %s" % (short, flag))
        cur = g[flag]
        g[flag] = (val not in ("0", "false", "False")) if isinstance(cur, bool) else type(cur)(val)


def sources():
    return sorted(glob.glob(os.path.join(CSRC, "*.hip")))


def build(force=False, verbose=False, out=None, defines=()):
    """Compile every HIP source into _build/libvst_hip.so for gfx950 (cross-compiles without a GPU).
    out/defines: developer variant builds (tools/build_variant.py)."""
    lib_path = out or os.path.join(BUILD, "libvst_hip.so")
    if out is None and any(d.split("=")[0] == "VST_DEV_VARIANT" for d in defines):
        raise ValueError("VST_DEV_VARIANT builds go to a variant path (tools/build_variant.py), never the product library")
    objdir = os.path.join(os.path.dirname(lib_path), "obj_" + os.path.basename(lib_path)[:-3])
    os.makedirs(objdir, exist_ok=True)
    srcs = sources()
    deps = srcs + glob.glob(os.path.join(CSRC, "*.h")) + [os.path.join(REPO, "include", "vst_hip.h"),
                                                          os.path.abspath(__file__)]
    if not force and os.path.exists(lib_path):
        if os.path.getmtime(lib_path) >= max(os.path.getmtime(d) for d in deps):
            return lib_path
    objs = []
    procs = []
    for s in srcs:
        o = os.path.join(objdir, os.path.basename(s) + ".o")
        objs.append(o)
        cmd = [HIPCC, "-O3", "-std=c++17", f"--offload-arch={ARCH}", "-fPIC", "-munsafe-fp-atomics",
               "-Wall", "-Wno-unused-function"] + FILE_FLAGS.get(os.path.basename(s), []) + \
            ["-D" + d for d in defines] + ["-c", s, "-o", o]
        if out is not None:  # developer variant builds only: extra compiler flags
            cmd[1:1] = os.environ.get("VST_VARIANT_HIPCC_FLAGS", "").split()
        procs.append((cmd, subprocess.Popen(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT)))
    for cmd, p in procs:
        out, _ = p.communicate()
        if p.returncode != 0:
            raise RuntimeError("hipcc failed: %s\n%s" % (" ".join(cmd), out.decode(errors="replace")))
        if verbose and out:
            print(out.decode(errors="replace"))
    tmp = lib_path + ".tmp"
    cmd = [HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", tmp] + objs
    r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT)
    if r.returncode != 0:
        raise RuntimeError("link failed: %s\n%s" % (" ".join(cmd), r.stdout.decode(errors="replace")))
    os.replace(tmp, lib_path)
    return lib_path


def load():
    """Return the loaded ctypes library; raises if it is missing (no CPU fallback exists)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise RuntimeError(
            f"libvst_hip.so not found at {LIB_PATH}; run __graft_entry__.build() (hipcc, gfx950)")
    lib = ctypes.CDLL(LIB_PATH)
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib


def exported_symbols():
    return list(SIGNATURES)


def check(rc, what=""):
    if rc != 0:
        msg = _lib.vst_last_error().decode(errors="replace") if _lib is not None else ""
        raise RuntimeError(f"libvst_hip {what} failed (status {rc}): {msg}")
