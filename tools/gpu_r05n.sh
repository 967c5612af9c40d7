#!/bin/bash
# Round-5: planes-only ResnetBlock backward chain (VST_APRE_BWD) and the StarGAN generator's phase / direct data
# gradients — op tests, model tests with APRE_BWD on, StarGAN tests, the StarGAN line, a same-box step A/B ($ARMS).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r05n}
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_ops.py -k "apre or pack_batch or skinny_split or conv4s2 or dgrad_refl_in" > $O/t_ops.log 2>&1 || { echo ops tests failed; tail -30 $O/t_ops.log; exit 1; }
tail -1 $O/t_ops.log
VST_APRE_BWD=1 timeout -k 10 300 python -u -m pytest -x -q --timeout 250 --timeout-method thread -m gpu tests/test_gpu_models.py > $O/t_models.log 2>&1 || { echo model tests failed; tail -30 $O/t_models.log; exit 1; }
tail -1 $O/t_models.log
timeout -k 10 400 python -u -m pytest -x -q --timeout 250 --timeout-method thread -m gpu tests/test_gpu_stargan.py tests/test_gpu_fullsize.py -k "stargan" > $O/t_sg.log 2>&1 || { echo stargan tests failed; tail -30 $O/t_sg.log; exit 1; }
tail -1 $O/t_sg.log
timeout -k 10 200 python3 tools/sgbench.py > $O/sg.log 2>&1 || { echo "sgbench failed"; tail -5 $O/sg.log; exit 1; }
echo "sg $(tail -1 $O/sg.log | grep -o '"ms_per_d_iteration": [0-9.]*')"
[ -n "$ARMS" ] && TAG=${TAG:-r05n}/ab bash tools/ab_step.sh
exit 0
