#!/bin/bash
# Round-5: the IN-backward partials in the ResnetBlock data gradient's epilogue (VST_DGRAD_EPI): its op tests,
# the full-size step vs the oracle with it on, the per-layer table + step trace at the current stamp (default
# route), then a same-box step A/B ($ARMS).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r05h}
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_ops.py -k "dgrad_refl_in" > $O/t_ops.log 2>&1 || { echo ops tests failed; tail -30 $O/t_ops.log; exit 1; }
tail -1 $O/t_ops.log
VST_DGRAD_EPI=1 timeout -k 10 300 python -u -m pytest -x -q --timeout 250 --timeout-method thread -m gpu tests/test_gpu_models.py -k "full_size_train_step" > $O/t_full.log 2>&1 || { echo full-size test failed; tail -30 $O/t_full.log; exit 1; }
tail -1 $O/t_full.log
python -c "import sys; sys.path.insert(0,'.'); import gbvst; print(gbvst._lib.source_stamp())" > $O/stamp.txt
timeout -k 10 240 python -u tools/layertable.py 3 > $O/layertable.jsonl 2> $O/layertable.err || { echo layertable failed; tail -20 $O/layertable.err; exit 1; }
tail -1 $O/layertable.jsonl
TAG=${TAG:-r05h}/trace bash tools/gpu_trace.sh > /dev/null || exit 1
[ -n "$ARMS" ] && TAG=${TAG:-r05h}/ab bash tools/ab_step.sh
exit 0
