# enrich kernel time vs symbol count at T = 10k (tail / ramp check)
set -o pipefail
cd $GRAFT_REPO_ROOT
for S in ${SS:-6144 12288 12500 13056 18432 25000 50000}; do
  timeout -k 10 300 python bench.py --symbols $S --no-shard --no-cpu-baseline --no-tick --no-breadth --no-rows --steps 10 | python -c "import json,sys; d=json.load(sys.stdin); r=d['roofline']; print('S=$S', round(r['kernel_ms'],4), 'ms', round(r['frac'],4), 'per12.5k', round(r['kernel_ms']*12500/$S,4))" || exit 1
done
