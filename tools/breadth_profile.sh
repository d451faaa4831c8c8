# C5 leg: bench line (breadth only) + rocprofv3 kernel stats of the same command.
# Usage: bash tools/breadth_profile.sh <tag>
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$1
mkdir -p $O
ARGS="--no-cpu-baseline --no-rows --no-tick --no-shard --steps 2 --warmup 1 --breadth-steps 5"
cd $R
timeout -k 10 600 python -u bench.py $ARGS > $O/bench.json 2> $O/bench.err || { echo BENCH_FAILED; tail $O/bench.err; exit 1; }
python -c "import json; d=json.load(open('$O/bench.json'))['breadth']; print(json.dumps(d))"
cd /tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 $R/bench.py $ARGS > /dev/null 2> $O/trace.err || { echo TRACE_FAILED; tail $O/trace.err; exit 1; }
rm -f $O/trace/run_kernel_trace.csv
head -12 $O/trace/run_kernel_stats.csv | cut -c1-200
