# Copy one round-profile tag (tools/round_profile.sh) and one row-profile tag
# (tools/row_profile.sh) from gpurun_out/ into profiles/ (tracked):
# bash tools/save_profiles.sh <round-tag> [<rows-tag>]
set -e
cd "$(dirname "$0")/.."
T=$1; R=$2
G=gpurun_out
if [ -n "$T" ] && [ -d $G/$T ]; then
  cp $G/$T/bench.json profiles/${T}_bench.json
  cp $G/$T/gpu_tests.log profiles/${T}_gpu_tests.log
  cp $G/$T/smoke.log profiles/${T}_smoke.log
  cp $G/$T/trace/run_kernel_stats.csv profiles/${T}_kernel_stats.csv
  cp $G/$T/trace_summary.txt profiles/${T}_trace_summary.txt
  cp $G/$T/pmc_traffic.json profiles/${T}_pmc_summary.json
fi
if [ -n "$R" ] && [ -d $G/$R ]; then
  mkdir -p profiles/$R
  cp $G/$R/rows_summary.json $G/$R/rows_summary.txt profiles/$R/
  for d in $G/$R/*/; do
    row=$(basename $d)
    [ -f $d/trace/run_kernel_stats.csv ] && cp $d/trace/run_kernel_stats.csv profiles/$R/${row}_kernel_stats.csv
  done
fi
