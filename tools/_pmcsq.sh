# SQ counter passes over one conv family of tools/kbench.py (KB=fprop|tconv|wgrad) -> gpurun_out/$TAG/
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; OUT=gpurun_out/${TAG:-pmcsq}; mkdir -p $OUT
P1="SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES"
P2="SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_SALU"
i=0
for P in "$P1" "$P2"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $P --output-format csv -d $OUT/sq_$i -o p -- python3 tools/kbench.py ${KB:-wgrad} 5 > $OUT/sq_$i.log 2>&1 || { echo "pmc fail $i"; tail -5 $OUT/sq_$i.log; exit 1; }
done
timeout -k 10 90 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt -o p -- python3 tools/kbench.py ${KB:-wgrad} 5 > $OUT/kt.log 2>&1 || { echo "kt fail"; exit 1; }
echo ok
