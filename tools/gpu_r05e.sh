#!/bin/bash
# Round-5: tile-kind sweep of the ConvTranspose / stride-2 families (VST_CONVT_TILE, VST_WG_KIND_S2):
# per arm the phase / wgrad parity tests, then the per-layer table.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r05e}
mkdir -p $O
for arm in ${ARMS:-default}; do
  if [ "$arm" = default ]; then envs=""; else envs="${arm//,/ }"; fi
  env $envs timeout -k 10 200 python -u -m pytest -x -q --timeout 100 --timeout-method thread -m gpu tests/test_gpu_ops.py -k "convT_phases or conv4s2 or (conv_fwd_dgrad_wgrad and auto) or wgrad_with_premade or fwd_cp_and_wgrad" > $O/t_$arm.log 2>&1 || { echo "tests failed $arm"; tail -20 $O/t_$arm.log; exit 1; }
  env $envs timeout -k 10 240 python -u tools/layertable.py 3 2> $O/lt_$arm.err | grep '^{' > $O/lt_$arm.jsonl || { echo "layertable failed $arm"; tail -20 $O/lt_$arm.err; exit 1; }
  echo "$arm $(tail -2 $O/t_$arm.log | head -1) $(tail -1 $O/lt_$arm.jsonl)"
done
