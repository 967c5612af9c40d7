"""Average SQ counters per dispatch of kernels matching a substring: sqsum.py <dir> [substring]."""
import csv
import glob
import sys
from collections import defaultdict

d, sub = sys.argv[1], (sys.argv[2] if len(sys.argv) > 2 else "conv")
vals = defaultdict(lambda: defaultdict(float))
names = {}
for f in glob.glob(d + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if sub in r["Kernel_Name"]:
            vals[r["Counter_Name"]][r["Dispatch_Id"]] += float(r["Counter_Value"])
            names[r["Dispatch_Id"]] = r["Kernel_Name"][:70]
for c, v in sorted(vals.items()):
    print("%-28s %.4g" % (c, sum(v.values()) / len(v)))
print(set(names.values()))
