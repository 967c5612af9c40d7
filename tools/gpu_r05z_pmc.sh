#!/bin/bash
# Round-5 final counters (after the last kernel change): rocprofv3 --pmc passes over the ResnetBlock conv ops, c0 and the
# warp (tools/profile_counters.sh), summarised into gpurun_out/r05z_pmc/r05z_conv_pmc.json (bench.py reads it from
# profiles/ when its source stamp matches).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
TAG=r05z_pmc OPS="fprop dgrad wgrad_pre wgrad c0 warp" bash tools/profile_counters.sh || exit 1
timeout -k 10 120 python3 tools/pmc_resblock.py gpurun_out/r05z_pmc gpurun_out/r05z_pmc/r05z 5 || exit 1
exit 0
