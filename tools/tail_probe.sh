# Tail-effect probe of the enrich launch: per-candle rate at symbol counts that
# fill whole rounds of resident workgroups (768 = 256 CUs x 3) vs 12 500.
set -o pipefail
cd $GRAFT_REPO_ROOT
for s in 12288 12500 13056 12500 12288; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-tick --no-breadth --no-rows --steps 20 --symbols $s | python -c "import json,sys; d=json.load(sys.stdin); print($s, round(d['roofline']['kernel_ms'],4), round(d['roofline']['frac'],4))" || exit 1
done
