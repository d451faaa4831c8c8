# enrich efficiency vs panel shape at fixed bytes (rounds vs kernel duration)
set -o pipefail
cd $GRAFT_REPO_ROOT
for sh in ${SHAPES:-12500x80000 100000x1250 12500x10000 100000x10000}; do
  S=${sh%x*}; T=${sh#*x}
  timeout -k 10 400 python bench.py --symbols $S --candles $T --no-shard --no-cpu-baseline --no-tick --no-breadth --no-rows --steps 5 | python -c "import json,sys; d=json.load(sys.stdin); r=d['roofline']; print('$sh', round(r['kernel_ms'],4), 'ms', round(r['frac'],4))" || exit 1
done
