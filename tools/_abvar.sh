# A/B library variants on the train-step bench: bash tools/_abvar.sh NAME1 NAME2 ... (lib_<NAME>.so
# from tools/build_variant.py; "base" = the in-tree library), two alternating passes
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/abv
for pass in 1 2; do
  for v in "$@"; do
    if [ "$v" = base ]; then L=""; else L=gan-based-video-style-transfer_amd/_build/variants/lib_$v.so; fi
    VST_LIB_VARIANT=$L timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-extras > gpurun_out/abv/$v.$pass.txt 2>&1 || { echo "fail $v"; tail -3 gpurun_out/abv/$v.$pass.txt; exit 1; }
    echo "$v" $(tail -1 gpurun_out/abv/$v.$pass.txt | cut -c60-110)
  done
done
