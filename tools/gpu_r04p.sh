bash tools/gpu_call.sh \
  "timeout -k 10 600 python3 -u -m pytest -x -v --timeout 500 --timeout-method thread tests/test_gpu_dp.py tests/test_gpu_fullsize.py -p no:cacheprovider" \
  "TAG=r04p_pmc OPS=\"fprop dgrad wgrad_pre wgrad c0 warp\" bash tools/profile_counters.sh" \
  "python3 tools/pmc_resblock.py gpurun_out/r04p_pmc profiles/r04p 5"
