# inference A/B: the ResnetBlock IN + ReLU in the second conv's A staging (VST_NRM_FWD=1, default)
# vs the apply pass (0); B=1 and B=16 at 256^2 and B=1 at 436x1024, alternating
for cfg in "1 256 256 60" "16 256 256 20" "1 436 1024 30"; do
  for r in 1 0 1 0; do echo -n "nrm=$r B H W reps=$cfg: "; VST_NRM_FWD=$r timeout -k 10 90 python3 tools/infbench.py $cfg || exit $?; done
done
