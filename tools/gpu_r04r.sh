bash tools/gpu_call.sh \
  "timeout -k 10 1000 python3 -u -m pytest -q --timeout 280 --timeout-method thread tests -m gpu -p no:cacheprovider"
