#!/bin/bash
# The committed bench line (default run, as the driver does) + the step kernel trace.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-final}
mkdir -p $OUT
timeout -k 10 600 python -u bench.py --steps 20 --warmup 5 > $OUT/bench.json 2> $OUT/bench.err || { echo bench failed; tail -20 $OUT/bench.err; exit 1; }
tail -c 400 $OUT/bench.json
TAG=${TAG:-final}_trace bash tools/gpu_trace.sh
