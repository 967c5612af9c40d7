bash tools/gpu_call.sh \
  "timeout -k 10 900 python3 -u -m pytest -x -q --timeout 280 --timeout-method thread tests -m gpu -p no:cacheprovider" \
  "TAG=r04q_trace bash tools/gpu_trace.sh" \
  "timeout -k 10 400 python3 bench.py > gpurun_out/r04q_bench.json"
