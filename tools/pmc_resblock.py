"""Summarise rocprofv3 counter passes over tools/kbench.py (fprop | dgrad | wgrad, KB_B frames of the
ResnetBlock shape, `reps` calls each) into profiles/<tag>_conv_pmc.json (read by bench.py's roofline
`traffic`) and a readable SQ summary.

usage: pmc_resblock.py <out_dir_of_pmc_runs> <profiles/tag> [reps]
Expected layout (tools/profile_counters.sh): <dir>/<op>_fetch, <op>_write, <op>_sq1, <op>_sq2, <op>_kt.
HBM bytes per call: FETCH_SIZE x 2 (the gfx950 wide-read correction, MI355X_MICROARCH.md HBM
section) + WRITE_SIZE, summed over every dispatch the op launches (dgrad: the 256x128 main + 64x64
tail launches; wgrad: the channel-major / bf16-plane copies, the GEMM, the split-K reduce + store).
"""
import csv
import glob
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

OPS = {"fprop": ("conv_fprop_bf_k",), "dgrad": ("conv_fprop_bf_k", "fprop_splitk_reduce_k", "dgrad_border_add_k", "dgrad_border5_add_k"),
       "wgrad": ("nhwc_to_cp", "conv_wgrad_bf_k", "wgrad_reduce_store_k", "slab_group_sum_k"),
       "wgrad_pre": ("conv_wgrad_bf_k", "wgrad_reduce_store_k", "slab_group_sum_k"),
       "wgrad_nhwc": ("conv_wgrad_nhwc_k", "wgrad_reduce_store_k", "slab_group_sum_k"),
       "warp": ("warp_fwd_k",), "c0": ("conv_c4_", "in_finalize_k")}
# the op's main GEMM dispatch (SQ metrics and its timing; the dgrad's 64x64 tail launch is excluded)
MAIN = {"fprop": "3>, true, 1, false, false>", "dgrad": "3>, true, 0, false, false>", "wgrad": "conv_wgrad_bf_k",
        "wgrad_pre": "conv_wgrad_bf_k", "wgrad_nhwc": "conv_wgrad_nhwc_k",
        "warp": "warp_fwd_k", "c0": "conv_c4_"}  # c0: the ring or the lock-step kernel
WARP_BYTES = 32 * 436 * 1024 * (8.0 * 64 + 8.0)  # bench.py warp_roofline: N*H*W*(4C gather + 8 flow + 4C write)


def counters(d, subs):
    vals = {}
    for f in glob.glob(d + "/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if any(s in r["Kernel_Name"] for s in subs):
                key = (r["Counter_Name"], r["Dispatch_Id"])
                vals[key] = vals.get(key, 0.0) + float(r["Counter_Value"])
    out = {}
    for (c, _), v in vals.items():
        out.setdefault(c, []).append(v)
    return out


def kernel_times(d, sub):
    t = []
    for f in glob.glob(d + "/**/*kernel_trace.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if sub in r["Kernel_Name"]:
                t.append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    return t


def main():
    d, tag = sys.argv[1], sys.argv[2]
    reps = int(sys.argv[3]) if len(sys.argv) > 3 else 5
    B = int(os.environ.get("KB_B", "8"))
    res, lines = {}, []
    sf = os.path.join(d, "source_stamp.txt")   # written on the GPU box by profile_counters.sh
    if os.path.exists(sf):
        stamp = open(sf).read().strip()
    else:
        from gbvst import _lib as _L
        stamp = _L.source_stamp()
    for op, subs in OPS.items():
        fetch = counters(os.path.join(d, op + "_fetch"), subs).get("FETCH_SIZE", [])
        write = counters(os.path.join(d, op + "_write"), subs).get("WRITE_SIZE", [])
        if not fetch or not write:
            continue
        fb, wb = 2 * sum(fetch) * 1024 / reps, sum(write) * 1024 / reps
        if op == "warp":
            alg = WARP_BYTES
        elif op == "c0":  # the 4-channel image read once + the 64-channel output written once + weight planes
            alg = 4.0 * B * 256 * 256 * (4 + 64) + 64 * 196 * 3 * 2
        else:
            alg = 4.0 * B * 64 * 64 * 256 * 2 + 256 * 2304 * 3 * 2
        t = kernel_times(os.path.join(d, op + "_kt"), MAIN[op])
        name = op if op in ("warp", "c0") else "resblock_" + op
        key = {"N": 32, "C": 64, "H": 436, "W": 1024} if op == "warp" else {"math": "bf16x6", "N": B}
        if op != "warp":  # the MFMA instruction of this build (bench.py matches records on it)
            import gbvst
            gbvst._lib.load()
            info = gbvst._lib.load().vst_build_info().decode()
            key["mfma"] = "v_mfma_f32_%s_bf16" % info.split("x6_mfma=")[1].split()[0]
        if op in ("fprop", "dgrad"):
            import gbvst
            from gbvst import ops
            gbvst._lib.load()
            # the reflect-pad-1 data gradient: the interior as the zero-pad-1 conv (+ the border GEMM)
            kind, ms = ops.conv_plan_fwd(B, 64, 64, 256, 256, 3, 3, 1, 1, 1, "bf16x6")
            ks = ops.conv_plan_fwd_tail(B, 64, 64, 256, 256, 3, 3, 1, 1, "bf16x6") if (ms and ops.FWD_SPLITK) else 0
            key.update(tile=kind, m_split=ms, ksplit=ks)
            if op == "dgrad":
                key["op"] = "dgrad_refl"  # bench.py's dgrad key
        res[name] = {"key": key, "source_stamp": stamp, "dispatches_per_call": len(fetch) / reps, "fetch_bytes": fb, "write_bytes": wb,
                     "hbm_bytes_per_launch": fb + wb, "algorithmic_bytes": alg,
                     "main_kernel_avg_us": round(sum(t) / len(t), 2) if t else None,
                     "note": "FETCH_SIZE x2 (gfx950 wide-read correction) + WRITE_SIZE, summed over the op's dispatches"}
        sq = counters(os.path.join(d, op + "_sq1"), (MAIN[op],))
        sq.update(counters(os.path.join(d, op + "_sq2"), (MAIN[op],)))
        lines.append("== %s (%s, N=%d): main kernel avg %s us over %d calls" % (op, MAIN[op], B, res[name]["main_kernel_avg_us"], reps))
        lines.append("   HBM per call: fetch %.1f MB + write %.1f MB = %.1f MB (algorithmic %.1f MB)" % (fb / 1e6, wb / 1e6, (fb + wb) / 1e6, alg / 1e6))
        for c in sorted(sq):
            v = sq[c]
            lines.append("   %-28s %.4g per dispatch" % (c, sum(v) / len(v)))
        if "SQ_WAVE_CYCLES" in sq and "SQ_WAIT_ANY" in sq:
            w = sum(sq["SQ_WAVE_CYCLES"])
            lines.append("   wait_any/wave_cycles %.3f  wait_inst_any/wave_cycles %.3f  active_inst_any/wave_cycles %.3f" % (
                sum(sq["SQ_WAIT_ANY"]) / w, sum(sq.get("SQ_WAIT_INST_ANY", [0])) / w, sum(sq.get("SQ_ACTIVE_INST_ANY", [0])) / w))
        if t:
            res[name]["achieved_GBps_main_kernel"] = round(alg / (sum(t) / len(t) * 1e-6) / 1e9, 1) if op == "warp" else None
        if "SQ_VALU_MFMA_BUSY_CYCLES" in sq and t and op != "warp":
            busy = sum(sq["SQ_VALU_MFMA_BUSY_CYCLES"]) / len(sq["SQ_VALU_MFMA_BUSY_CYCLES"])
            dur = sum(t) / len(t) * 1e-6
            lines.append("   MFMA busy fraction (busy cycles / (1024 SIMDs x 2.4 GHz x avg duration)): %.3f" % (busy / (1024 * 2.4e9 * dur)))
            res[name]["mfma_busy_frac_nominal_clock"] = round(busy / (1024 * 2.4e9 * dur), 4)
            if "SQ_WAVE_CYCLES" in sq and "SQ_WAVES" in sq:
                # SQ_WAVE_CYCLES counts quad-cycles (MI355X_MICROARCH.md); a wave lives ~the whole
                # kernel (one block per CU, one round), so this is MFMA busy vs cycles at the real clock
                life = 4.0 * sum(sq["SQ_WAVE_CYCLES"]) / sum(sq["SQ_WAVES"])
                clk = life / dur
                lines.append("   MFMA busy vs wave-lifetime cycles: %.3f (effective clock %.2f GHz)" % (busy / (1024 * life), clk / 1e9))
                res[name]["mfma_busy_frac_actual_clock"] = round(busy / (1024 * life), 4)
                res[name]["effective_clock_GHz"] = round(clk / 1e9, 3)
    json.dump(res, open(tag + "_conv_pmc.json", "w"), indent=1)
    open(tag + "_conv_sq.txt", "w").write("\n".join(lines) + "\n")
    print("\n".join(lines))


if __name__ == "__main__":
    main()
