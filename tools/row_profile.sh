# Per-row rocprofv3 evidence for DESIGN §6 / bench `rows`: for each row, one
# kernel-trace + stats pass and four PMC passes (two SQ groups, FETCH_SIZE,
# WRITE_SIZE; torch's own kernels excluded) of `python tools/row_prof.py ROW`,
# then tools/row_summary.py -> gpurun_out/<tag>/rows_summary.json.
# Usage: bash tools/row_profile.sh <tag> ROW [ROW ...]   (S x T via ROW_S / ROW_T)
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
TAG=$1; shift
O=$R/gpurun_out/$TAG
mkdir -p $O
cd /tmp
EXC='at::native|at_cuda_detail|rocprim|elementwise'
for row in "$@"; do
  D=$O/$row
  mkdir -p $D
  timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $D/trace -o run -- python3 $R/tools/row_prof.py $row $ROW_S $ROW_T > $D/trace.log 2>&1 || { echo "$row trace failed"; tail -3 $D/trace.log; exit 1; }
  i=0
  for grp in "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU" \
             "SQ_INSTS_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE" \
             "FETCH_SIZE" "WRITE_SIZE"; do
    i=$((i+1))
    timeout -s KILL 120 rocprofv3 --pmc $grp --kernel-exclude-regex "$EXC" --output-format csv -d $D/p$i -o run -- python3 $R/tools/row_prof.py $row $ROW_S $ROW_T > $D/p$i.log 2>&1 || { echo "$row pmc pass $i failed"; tail -3 $D/p$i.log; exit 1; }
  done
  echo "$row: $(tail -1 $D/trace.log)"
done
cd $R
python tools/row_summary.py $O "$@" > $O/rows_summary.txt && cat $O/rows_summary.txt
