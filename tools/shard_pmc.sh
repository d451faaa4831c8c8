# Enrich kernel at the C4 shard (12.5k x 10k) against the 100k headline
# (VERDICT r5 next #3): kernel trace + PMC passes — HBM bytes (FETCH_SIZE x2,
# WRITE_SIZE), L2 hit / miss and the L2 -> DRAM read / write credit stalls,
# the SQ occupancy / wait counters — for the padded-pitch outputs (default)
# and contiguous [S, T] outputs at the shard, and the padded headline.
# Usage: bash tools/shard_pmc.sh <tag>  -> gpurun_out/<tag>/<case>/...
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$1
mkdir -p $O
cd /tmp
EXC='at::native|at_cuda_detail|rocprim|elementwise'
for case in "enrich 12500" "enrich_flat 12500" "enrich 100000"; do
  set -- $case
  D=$O/${1}_$2
  mkdir -p $D
  timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $D/trace -o run -- python3 $R/tools/row_prof.py $1 $2 10000 > $D/trace.log 2>&1 || { echo "$case trace failed"; tail -3 $D/trace.log; exit 1; }
  i=0
  for grp in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum TCC_EA0_WRREQ_DRAM_CREDIT_STALL_sum TCC_EA0_RDREQ_DRAM_CREDIT_STALL_sum" \
             "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU GRBM_GUI_ACTIVE"; do
    i=$((i+1))
    timeout -s KILL 120 rocprofv3 --pmc $grp --kernel-exclude-regex "$EXC" --output-format csv -d $D/p$i -o run -- python3 $R/tools/row_prof.py $1 $2 10000 > $D/p$i.log 2>&1 || { echo "$case pmc pass $i failed"; tail -3 $D/p$i.log; exit 1; }
  done
  echo "$case: $(tail -1 $D/trace.log)"
done
cd $R
python tools/shard_summary.py $O > $O/shard_summary.txt && cat $O/shard_summary.txt
