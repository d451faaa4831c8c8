# enrich kernel time at 12.5k x 10k vs the number of timed steps (clock / warm-state check)
set -o pipefail
cd $GRAFT_REPO_ROOT
for st in ${STEPS_LIST:-5 20 100}; do
  timeout -k 10 300 python bench.py --symbols ${S:-12500} --no-shard --no-cpu-baseline --no-tick --no-breadth --no-rows --steps $st --warmup ${W:-3} | python -c "import json,sys; d=json.load(sys.stdin); r=d['roofline']; print('steps=$st', round(r['kernel_ms'],4), 'ms', round(r['frac'],4))" || exit 1
done
