# c0 (4-channel 7x7 first conv) A/B: the row-ring kernel (default) vs the lock-step one (VST_C4_RING=0)
for m in in plain; do
  for r in 1 0 1 0; do echo -n "ring=$r: "; VST_C4_RING=$r KB_MODE=$m timeout -k 10 60 python3 tools/kbench_c0.py || exit $?; done
done
