"""Summarise a rocprofv3 --kernel-trace CSV: per (kernel, grid) total/avg time, per-step share."""
import csv
import sys
from collections import defaultdict

path = sys.argv[1]
steps = float(sys.argv[2]) if len(sys.argv) > 2 else 1.0
top = int(sys.argv[3]) if len(sys.argv) > 3 else 40
rows = list(csv.DictReader(open(path)))
d = defaultdict(list)
for r in rows:
    name = r["Kernel_Name"].split("(")[0].replace("void ", "")  # full template name
    key = "%s g=%s,%s,%s b=%s" % (name, r["Grid_Size_X"], r["Grid_Size_Y"], r["Grid_Size_Z"], r["Workgroup_Size_X"])
    d[key].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
tot = sum(sum(v) for v in d.values())
print("total kernel time %.1f ms  (%.2f ms/step over %g steps)" % (tot / 1e6, tot / 1e6 / steps, steps))
for k, v in sorted(d.items(), key=lambda kv: -sum(kv[1]))[:top]:
    print("%-110s n=%5d avg=%8.1fus tot/step=%7.2fms %5.1f%%" % (k, len(v), sum(v) / len(v) / 1e3,
                                                                 sum(v) / 1e6 / steps, 100 * sum(v) / tot))
