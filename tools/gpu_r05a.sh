#!/bin/bash
# Round-5 baseline: the per-layer conv table and the step kernel trace at the current source stamp.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r05a}
mkdir -p $O
python -c "import sys; sys.path.insert(0,'.'); import gbvst; print(gbvst._lib.source_stamp())" > $O/stamp.txt
timeout -k 10 240 python -u tools/layertable.py 3 > $O/layertable.jsonl 2> $O/layertable.err || { echo layertable failed; tail -20 $O/layertable.err; exit 1; }
tail -1 $O/layertable.jsonl
TAG=${TAG:-r05a}/trace bash tools/gpu_trace.sh
