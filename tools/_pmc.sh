cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; OUT=gpurun_out/pmc1; mkdir -p $OUT
P1="SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES"
P2="SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_SALU"
for m in bf16x3 bf16x6; do
 for k in fprop; do
  i=0
  for P in "$P1" "$P2"; do
   i=$((i+1))
   VST_CONV_MATH=$m timeout -s KILL 90 rocprofv3 --pmc $P --output-format csv -d $OUT/${m}_${k}_$i -o p -- python3 tools/kbench.py $k 5 > $OUT/${m}_${k}_$i.log 2>&1 || { echo "pmc fail $m $k $i"; tail -5 $OUT/${m}_${k}_$i.log; exit 1; }
  done
 done
done
echo ok
