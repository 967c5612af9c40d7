#!/bin/bash
# A/B of developer variant builds (tools/build_variant.py -> _build/variants/lib_<name>.so) on the
# ResnetBlock conv kernels: tools/kbench_time.py per variant, two interleaved rounds.
# usage: VARIANTS="lf pr ..." TAG=... tools/ab_variants.sh
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-ab}
mkdir -p $OUT
V=_build_dummy
for round in 1 2; do
  for v in default $VARIANTS; do
    if [ "$v" = default ]; then unset VST_LIB_VARIANT; else export VST_LIB_VARIANT=gan-based-video-style-transfer_amd/_build/variants/lib_$v.so; fi
    KB_B=${KB_B:-8} timeout -k 10 120 python -u tools/kbench_time.py >> $OUT/ab.jsonl 2> $OUT/ab_$v.err
    rc=$?
    if [ $rc -ne 0 ]; then echo "variant $v failed rc=$rc"; tail -5 $OUT/ab_$v.err; exit $rc; fi
    tail -1 $OUT/ab.jsonl
  done
done
unset VST_LIB_VARIANT
echo ab done
