#!/bin/bash
# Counter passes over the ResnetBlock conv ops (tools/kbench.py, N=8, bf16x6) for the roofline
# record: FETCH_SIZE and WRITE_SIZE in separate rocprofv3 --pmc runs (TCC budget), two SQ passes
# (8 counters each), one kernel-trace pass.  Writes gpurun_out/$TAG/; then tools/pmc_resblock.py.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-pmc}
mkdir -p $OUT
# the kernel-source stamp of the code being profiled (tools/pmc_resblock.py stores it in the record)
python3 -c "import sys; sys.path.insert(0, '.'); from gbvst import _lib; print(_lib.source_stamp())" > $OUT/source_stamp.txt || exit 1
SQ1="SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES"
SQ2="SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_SALU"
for op in ${OPS:-fprop dgrad wgrad_nhwc wgrad_pre c0 warp}; do
  for pass in fetch write sq1 sq2; do
    case $pass in fetch) C=FETCH_SIZE;; write) C=WRITE_SIZE;; sq1) C=$SQ1;; sq2) C=$SQ2;; esac
    VST_CONV_MATH=bf16x6 timeout -s KILL 90 rocprofv3 --pmc $C --output-format csv -d $OUT/${op}_$pass -o p -- python3 tools/kbench.py $op 5 > $OUT/${op}_$pass.log 2>&1 || { echo "pmc fail $op $pass"; tail -5 $OUT/${op}_$pass.log; exit 1; }
  done
  VST_CONV_MATH=bf16x6 timeout -k 10 90 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/${op}_kt -o p -- python3 tools/kbench.py $op 5 > $OUT/${op}_kt.log 2>&1 || { echo "kt fail $op"; exit 1; }
done
echo counters done
