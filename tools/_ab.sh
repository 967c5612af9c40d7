set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/ab10; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_models.py tests/test_gpu_c3.py tests/test_gpu_train.py tests/test_library_ops.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { echo pytest fail; grep -E "FAIL|Error|assert" $O/pytest.log | head -30; tail -5 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for v in 1 0 1 0; do
  set -- $v
  VST_FWD_SPLITK=$1 timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-extras > $O/bench_$1.json 2>/dev/null || { echo bench fail; exit 1; }
  python -c "import json,sys; d=json.loads(open('$O/bench_$1.json').read().strip().splitlines()[-1]); print('splitk=$1', d['value'], d['ms_per_step'])"
done
