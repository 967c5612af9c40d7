#!/bin/bash
# SQ counter passes over tools/kbench_tap64.py (separate rocprofv3 --pmc runs) + a kernel trace.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-pmc_tap64}
mkdir -p $OUT
SQ1="SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES"
SQ2="SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_MFMA SQ_ACTIVE_INST_MISC SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS"
python3 tools/kbench_tap64.py 10 > $OUT/time.txt 2>&1 || exit 1
cat $OUT/time.txt | tail -1
for pass in sq1 sq2 fetch; do
  case $pass in sq1) C=$SQ1;; sq2) C=$SQ2;; fetch) C=FETCH_SIZE;; esac
  timeout -s KILL 60 rocprofv3 --pmc $C --output-format csv -d $OUT/$pass -o p -- python3 tools/kbench_tap64.py 5 > $OUT/$pass.log 2>&1 || { echo "pmc fail $pass"; tail -5 $OUT/$pass.log; exit 1; }
done
python3 - $OUT <<'PY'
import csv, glob, sys
d = sys.argv[1]
for p in ("sq1", "sq2", "fetch"):
    vals = {}
    for f in glob.glob(d + "/" + p + "/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if "tap64" in r["Kernel_Name"]:
                vals.setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
    for k, v in sorted(vals.items()):
        print("%-26s %.4g per dispatch" % (k, sum(v) / len(v)))
PY
