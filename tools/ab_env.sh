#!/bin/bash
# Same-box step A/B of an environment switch: bench.py --no-extras --no-cpu-baseline, alternating
# the two settings ROUNDS times.  usage: AB_VAR=VST_X AB_A=0 AB_B=1 TAG=.. bash tools/ab_env.sh
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-abenv}
mkdir -p $OUT
for r in $(seq 1 ${ROUNDS:-2}); do
  for v in "$AB_A" "$AB_B"; do
    env $AB_VAR=$v timeout -k 10 200 python -u bench.py --steps ${STEPS:-20} --warmup 5 --no-extras --no-cpu-baseline > $OUT/b_${v}_$r.json 2> $OUT/b_${v}_$r.err
    rc=$?
    if [ $rc -ne 0 ]; then echo "bench $AB_VAR=$v failed rc=$rc"; tail -5 $OUT/b_${v}_$r.err; exit $rc; fi
    tail -1 $OUT/b_${v}_$r.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$AB_VAR=$v', d['ms_per_step'], d['value'])"
  done
done
