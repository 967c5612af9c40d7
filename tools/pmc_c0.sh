#!/bin/bash
# rocprofv3 counter passes + kernel trace over tools/kbench_c0.py (the 4-channel 7x7 forward).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-pmc_c0}
mkdir -p $OUT
SQ1="SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES"
SQ2="SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_SALU"
for pass in sq1 sq2 grbm; do
  case $pass in sq1) C=$SQ1;; sq2) C=$SQ2;; grbm) C="GRBM_GUI_ACTIVE GRBM_COUNT";; esac
  timeout -s KILL 90 rocprofv3 --pmc $C --output-format csv -d $OUT/$pass -o p -- python3 tools/kbench_c0.py > $OUT/$pass.log 2>&1 || { echo "pmc fail $pass"; tail -5 $OUT/$pass.log; exit 1; }
done
timeout -k 10 90 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt -o p -- python3 tools/kbench_c0.py > $OUT/kt.log 2>&1 || { echo "kt fail"; exit 1; }
echo counters done
