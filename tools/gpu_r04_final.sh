# round-4 final measurements (after the last kernel change): counters at the current source stamp, the
# full GPU suite, smoke(), step and inference traces, the bench line
bash tools/gpu_call.sh \
  "TAG=r04f5_pmc OPS=\"fprop dgrad wgrad_pre wgrad c0 warp\" bash tools/profile_counters.sh" \
  "timeout -k 10 900 python3 -u -m pytest -q --timeout 280 --timeout-method thread tests -m gpu -p no:cacheprovider" \
  "timeout -k 10 300 python3 -c 'import __graft_entry__ as g; g.smoke(); print(\"smoke ok\")'" \
  "TAG=r04f5_trace bash tools/gpu_trace.sh" \
  "TAG=r04f5_inf bash tools/gpu_inftrace.sh" \
  "timeout -k 10 400 python3 bench.py > gpurun_out/r04f5_bench.json"
