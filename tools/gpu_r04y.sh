# round-4 final measurements: counters (fresh stamp), full GPU suite, step trace, inference traces, bench
bash tools/gpu_call.sh \
  "TAG=r04y_pmc OPS=\"fprop dgrad wgrad_pre wgrad c0 warp\" bash tools/profile_counters.sh" \
  "timeout -k 10 900 python3 -u -m pytest -q --timeout 280 --timeout-method thread tests -m gpu -p no:cacheprovider" \
  "TAG=r04y_trace bash tools/gpu_trace.sh" \
  "TAG=r04y_inf bash tools/gpu_inftrace.sh" \
  "timeout -k 10 400 python3 bench.py > gpurun_out/r04y_bench.json"
