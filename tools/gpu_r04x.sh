V=$GRAFT_REPO_ROOT/gan-based-video-style-transfer_amd/_build/variants
ARMS="default VST_LIB_VARIANT=$V/lib_fwdonly.so VST_LIB_VARIANT=$V/lib_nog.so" TAG=r04x_glds_step bash tools/ab_step.sh
