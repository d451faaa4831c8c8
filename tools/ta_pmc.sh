# TA / TD busy of one row's kernels (is the uncoalesced chunk addressing the
# slide kernels' limiter?): bash tools/ta_pmc.sh <tag> <row>
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$1/$2
mkdir -p $O
cd /tmp
EXC='at::native|at_cuda_detail|rocprim|elementwise'
i=0
for grp in "TA_BUSY_avr TA_BUSY_max GRBM_GUI_ACTIVE" "TD_BUSY_avr TD_BUSY_max GRBM_GUI_ACTIVE" "TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp --kernel-exclude-regex "$EXC" --output-format csv -d $O/t$i -o run -- python3 $R/tools/row_prof.py $2 > $O/t$i.log 2>&1 || { echo "pass $i failed"; tail -3 $O/t$i.log; exit 1; }
done
echo TA_PMC_DONE
