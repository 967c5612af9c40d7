set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/ab11; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_models.py -m gpu -x -q --timeout 120 --timeout-method thread -k "fold_instnorm or production or full_size" > $O/pytest.log 2>&1 || { echo pytest fail; tail -20 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for v in 1 0 1 0; do
  VST_FOLD_IN=$v timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-extras > $O/bench_$v.json 2>/dev/null || { echo bench fail; exit 1; }
  python -c "import json,sys; d=json.loads(open('$O/bench_$v.json').read().strip().splitlines()[-1]); print('fold_in=$v', d['value'], d['ms_per_step'])"
done
