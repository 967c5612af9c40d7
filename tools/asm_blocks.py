"""Developer: per-basic-block summary of one kernel in a hipcc -S listing (MFMAs, global loads,
vmcnt waits, barriers, branches) and its register counts.  usage: asm_blocks.py FILE.s SUBSTRING...
(every kernel whose mangled name contains all substrings)."""
import re
import sys

src = open(sys.argv[1]).read().split("\n")
keys = sys.argv[2:]
heads = [i for i, l in enumerate(src) if re.match(r"^_Z\S*:", l) and all(k in l.split(":")[0] for k in keys)]
for h in heads:
    name = src[h].split(":")[0]
    end = next(i for i in range(h, len(src)) if src[i].startswith("\t.size\t" + name))
    print(name)
    cur = None
    for l in src[h:end]:
        if re.match(r"^\.LBB", l):
            if cur:
                print("  ", cur)
            cur = {"blk": l.split(":")[0], "mfma": 0, "gload": 0, "vmcnt0": 0, "vmcnt": 0, "bar": 0, "br": 0,
                   "ds_r": 0, "ds_w": 0}
        elif cur is not None:
            cur["mfma"] += "v_mfma" in l
            cur["gload"] += "global_load" in l or "buffer_load" in l
            if "s_waitcnt" in l and "vmcnt" in l:
                cur["vmcnt0" if "vmcnt(0)" in l else "vmcnt"] += 1
            cur["bar"] += "s_barrier" in l
            cur["br"] += bool(re.search(r"\ts_c?branch", l))
            cur["ds_r"] += "ds_read" in l
            cur["ds_w"] += "ds_write" in l
    if cur:
        print("  ", cur)
    meta = [l.strip() for l in src[end:end + 40] if re.search(r"(vgpr|sgpr|agpr)_count|ScratchSize|Occupancy", l)]
    print("  ", meta[:6])
