# c0 ring kernel: product vs developer variants (tools/build_variant.py), plain mode (no IN partials)
V=$GRAFT_REPO_ROOT/gan-based-video-style-transfer_amd/_build/variants
for r in 1 2; do
  echo -n "product: "; KB_MODE=plain timeout -k 10 60 python3 tools/kbench_c0.py || exit $?
  for v in $(ls $V | sed -n 's/^lib_\(.*\)\.so$/\1/p'); do echo -n "$v: "; KB_MODE=plain VST_LIB_VARIANT=$V/lib_$v.so timeout -k 10 60 python3 tools/kbench_c0.py || exit $?; done
done
