cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out/ksl
export VST_LIB_VARIANT=gan-based-video-style-transfer_amd/_build/variants/lib_ksl.so
TAG=pmcksl bash tools/_pmc8.sh || exit 1
unset VST_LIB_VARIANT
bash tools/_abvar.sh base ksl
