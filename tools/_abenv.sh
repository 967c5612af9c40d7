# A/B an environment toggle: bash tools/_abenv.sh VAR  (runs bench with VAR=1, VAR=0, VAR=1, VAR=0)
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/abe
for v in 1 0 1 0; do
  env $1=$v timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-extras > gpurun_out/abe/$v.txt 2>&1 || { echo "fail $v"; tail -3 gpurun_out/abe/$v.txt; exit 1; }
  echo "$1=$v" $(tail -1 gpurun_out/abe/$v.txt | cut -c60-110)
done
