# A/B: bench (no extras) with the main library and each _build/variants/lib_<name>.so given as args
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/ab
for v in main "$@" main; do
  if [ $v = main ]; then unset VST_LIB_VARIANT; else export VST_LIB_VARIANT=$PWD/gan-based-video-style-transfer_amd/_build/variants/lib_$v.so; fi
  timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-extras > gpurun_out/ab/$v.txt 2>&1 || { echo "fail $v"; tail -3 gpurun_out/ab/$v.txt; exit 1; }
  echo $v $(tail -1 gpurun_out/ab/$v.txt | cut -c1-120)
done
