# HBM traffic of the C5 leg's pass-1 kernel at the bench's breadth shape
# (100k x 10k): FETCH_SIZE and WRITE_SIZE passes of the breadth-only bench
# command -> gpurun_out/<tag>/pmc_traffic.json (tools/pmc_summary.py,
# kernel "context_partials"). Usage: bash tools/breadth_pmc.sh <tag>
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$1
mkdir -p $O/pmc
ARGS="--no-cpu-baseline --no-rows --no-tick --no-shard --steps 1 --warmup 1 --breadth-steps 2"
cd /tmp
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 300 rocprofv3 --pmc $grp --output-format csv -d $O/pmc/p$i -o run -- python3 $R/bench.py $ARGS > $O/pmc/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $O/pmc/p$i.log; exit 1; }
done
cd $R
python tools/pmc_summary.py $O/pmc context_partials $O/pmc_traffic.json $1 1000000000 > /dev/null
python -c "import json; d=json.load(open('$O/pmc_traffic.json'))['context_partials']; print('context_partials traffic/launch', d['bytes_per_launch'], 'x alg', d['bytes_per_launch'] / 24e9)"
