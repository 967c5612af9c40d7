set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${TAG:-prof}; mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o prof -- python3 bench.py --steps 7 --warmup 3 --no-cpu-baseline --no-extras > $O/prof.log 2>&1 || { echo prof failed; tail -20 $O/prof.log; exit 1; }
echo done
