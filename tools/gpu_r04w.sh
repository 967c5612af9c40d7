bash tools/gpu_call.sh \
  "timeout -k 10 400 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_ops.py tests/test_gpu_models.py -p no:cacheprovider" \
  "VARIANTS=nog TAG=r04w_glds bash tools/ab_variants.sh" \
  "ARMS=\"default VST_LIB_VARIANT=$GRAFT_REPO_ROOT/gan-based-video-style-transfer_amd/_build/variants/lib_nog.so\" TAG=r04w_glds_step bash tools/ab_step.sh"
