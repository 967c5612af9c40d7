# kernel-trace the train-step bench with a library variant: VAR=<name> TAG=<dir> bash tools/_profvar.sh
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; OUT=gpurun_out/${TAG:-pv}; mkdir -p $OUT
export VST_LIB_VARIANT=gan-based-video-style-transfer_amd/_build/variants/lib_$VAR.so
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o prof -- python3 bench.py --steps 7 --warmup 3 --no-cpu-baseline --no-extras > $OUT/prof.log 2>&1 || { echo prof failed; tail -20 $OUT/prof.log; exit 1; }
echo done
