#!/bin/bash
# StarGAN kernel traces with / without VST_SG_DIRECT (kernel-time totals per D iteration) + the Johnson step trace.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
TAG=r05u/sg_direct bash tools/gpu_sgtrace.sh > /dev/null || exit 1
VST_SG_DIRECT=0 TAG=r05u/sg_autograd bash tools/gpu_sgtrace.sh > /dev/null || exit 1
head -1 gpurun_out/r05u/sg_direct/sg_summary.txt; head -1 gpurun_out/r05u/sg_autograd/sg_summary.txt
TAG=r05u/js bash tools/gpu_jstrace.sh > /dev/null || exit 1
head -12 gpurun_out/r05u/js/js_summary.txt | cut -c1-200
exit 0
