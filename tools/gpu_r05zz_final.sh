#!/bin/bash
# Round-5 final set, second take (after the RAFT / reduce-store kernel-source changes): the PMC passes (the bench's
# traffic record must carry the running sources' stamp), copied into profiles/ on the box before the bench runs, then
# the GPU suite, smoke(), the step / inference traces and the bench line.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
bash tools/gpu_r05z_pmc.sh > gpurun_out/r05z_pmc.log 2>&1 || { echo pmc failed; tail -20 gpurun_out/r05z_pmc.log; exit 1; }
cp gpurun_out/r05z_pmc/r05z_conv_pmc.json gpurun_out/r05z_pmc/r05z_conv_sq.txt profiles/ || exit 1
bash tools/gpu_r05z_final.sh
