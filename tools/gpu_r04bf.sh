bash tools/gpu_call.sh \
  "timeout -k 10 400 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_ops.py tests/test_gpu_models.py -p no:cacheprovider" \
  "ARMS=\"default VST_BORDER_FUSE=0\" TAG=r04bf_step bash tools/ab_step.sh"
