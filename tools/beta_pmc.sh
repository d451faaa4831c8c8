# PMC passes over tools/beta_prof.py (the a11 beta/corr kernel at 12.5k x 2k)
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd /tmp
i=0
for grp in "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU" \
           "SQ_INSTS_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM SQ_ACTIVE_INST_MISC" \
           "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $grp --output-format csv -d $R/gpurun_out/beta_pmc/p$i -o run -- python3 $R/tools/beta_prof.py > $R/gpurun_out/beta_pmc/p$i.log 2>&1 || { echo "pass $i failed"; tail -3 $R/gpurun_out/beta_pmc/p$i.log; exit 1; }
done
echo BETA_PMC_DONE
