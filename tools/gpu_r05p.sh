#!/bin/bash
# Round-5: StarGAN generator ConvTranspose forwards on phase convs + first-conv data gradient on the tap route — tests,
# the StarGAN line, its trace.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r05p}
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 250 --timeout-method thread -m gpu tests/test_gpu_stargan.py tests/test_gpu_fullsize.py tests/test_gpu_ops.py -k "stargan" > $O/t_sg.log 2>&1 || { echo stargan tests failed; tail -30 $O/t_sg.log; exit 1; }
tail -1 $O/t_sg.log
for arm in; do
  if [ "$arm" = default ]; then envs=""; else envs="$arm"; fi
  env $envs timeout -k 10 200 python3 tools/sgbench.py > $O/sg_$arm.log 2>&1 || { echo "sgbench $arm failed"; tail -5 $O/sg_$arm.log; exit 1; }
  echo "$arm $(tail -1 $O/sg_$arm.log | grep -o '"ms_per_d_iteration": [0-9.]*')"
done
for k in 0 1 2 0 1 2; do VST_PACK_KERNEL=$k timeout -k 10 120 python3 tools/packbench.py 2> $O/pb.err || { echo packbench failed; tail -5 $O/pb.err; exit 1; }; done
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_ops.py -k "pack_batch or phase_packs" > $O/t_pack.log 2>&1 || { echo pack tests failed; tail -30 $O/t_pack.log; exit 1; }
tail -1 $O/t_pack.log
exit 0
