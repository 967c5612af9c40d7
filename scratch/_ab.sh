set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/ab15; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py tests/test_library_ops.py tests/test_gpu_style.py -m gpu -x -q --timeout 120 --timeout-method thread -k "wgrad or gram or conv or style" > $O/pytest.log 2>&1 || { echo pytest fail; grep -E "FAIL|Error|assert" $O/pytest.log | head -30; tail -5 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
V=gan-based-video-style-transfer_amd/_build/variants
for v in default red0 default red0; do
  if [ $v = default ]; then L=""; else L=$V/lib_$v.so; fi
  VST_LIB_VARIANT=$L timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-extras > $O/bench_$v.json 2>/dev/null || { echo bench fail; exit 1; }
  python -c "import json,sys; d=json.loads(open('$O/bench_$v.json').read().strip().splitlines()[-1]); print('$v', d['value'], d['ms_per_step'])"
done
