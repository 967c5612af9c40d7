#!/bin/bash
# Round-5: pre-split A operands (VST_APRE) — op tests, the full-size step vs the oracle with it on, the pack batch
# test, then a same-box step A/B ($ARMS) and the StarGAN line.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r05l}
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_ops.py -k "apre or pack_batch or phase_packs or conv4s2 or dgrad_refl_in" > $O/t_ops.log 2>&1 || { echo ops tests failed; tail -30 $O/t_ops.log; exit 1; }
tail -1 $O/t_ops.log
VST_APRE=1 timeout -k 10 300 python -u -m pytest -x -q --timeout 250 --timeout-method thread -m gpu tests/test_gpu_models.py > $O/t_models.log 2>&1 || { echo model tests failed; tail -30 $O/t_models.log; exit 1; }
tail -1 $O/t_models.log
timeout -k 10 200 python3 tools/sgbench.py > $O/sg.log 2>&1 || { echo "sgbench failed"; tail -5 $O/sg.log; exit 1; }
echo "sg $(tail -1 $O/sg.log | grep -o '"ms_per_d_iteration": [0-9.]*')"
[ -n "$ARMS" ] && TAG=${TAG:-r05l}/ab bash tools/ab_step.sh
exit 0
