bash tools/gpu_call.sh \
  "timeout -k 10 300 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_ops.py -k \"c4_dgrad or c4_direct\" tests/test_gpu_models.py -p no:cacheprovider" \
  "ARMS=\"default VST_C4_DGRAD=0\" TAG=r04z_c4dgrad_step bash tools/ab_step.sh"
