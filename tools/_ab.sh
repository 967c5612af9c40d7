set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/ab14; mkdir -p $O
true
true
V=gan-based-video-style-transfer_amd/_build/variants
for v in default epi0 default epi0; do
  if [ $v = default ]; then L=""; else L=$V/lib_$v.so; fi
  VST_LIB_VARIANT=$L timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-extras > $O/bench_$v.json 2>/dev/null || { echo bench fail; exit 1; }
  python -c "import json,sys; d=json.loads(open('$O/bench_$v.json').read().strip().splitlines()[-1]); print('$v', d['value'], d['ms_per_step'])"
done
