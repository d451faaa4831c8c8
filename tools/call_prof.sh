# rocprofv3 kernel trace of tools/call_prof.py <name>; prints the per-kernel mean (us) table
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd /tmp
for n in $NAMES; do
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/callprof_$n -o run -- python3 $R/tools/call_prof.py $n > $R/gpurun_out/callprof_$n.log 2>&1 || { echo "prof $n failed"; tail -3 $R/gpurun_out/callprof_$n.log; exit 1; }
  grep " ms " $R/gpurun_out/callprof_$n.log
  f=$(find $R/gpurun_out/callprof_$n -name "*kernel_stats.csv" | head -1)
  python3 -c "
import csv,sys
rows=list(csv.DictReader(open('$f')))
for r in sorted(rows, key=lambda r: -float(r['TotalDurationNs']))[:8]:
    print('  %-70s calls=%s avg_us=%.1f' % (r['Name'][:70], r['Calls'], float(r['AverageNs'])/1000))
"
done
