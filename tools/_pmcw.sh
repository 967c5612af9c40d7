# FETCH/WRITE of the ResnetBlock wgrad (rk) at KB_B=8 -> gpurun_out/$TAG/pmcw.json
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; OUT=gpurun_out/${TAG:-pmcw}; mkdir -p $OUT
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc_f -o p -- python3 tools/kbench.py wgrad 5 > $OUT/pmc_f.log 2>&1 || { echo pmc fetch failed; tail -5 $OUT/pmc_f.log; exit 1; }
timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pmc_w -o p -- python3 tools/kbench.py wgrad 5 > $OUT/pmc_w.log 2>&1 || { echo pmc write failed; tail -5 $OUT/pmc_w.log; exit 1; }
python3 tools/pmc_conv.py $OUT/pmc_f $OUT/pmc_w $OUT/pmcw.json conv_wgrad_rk_k
