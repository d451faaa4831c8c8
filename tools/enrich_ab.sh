# GPU A/B of the enrich kernel's launch mode: headline (100k x 10k) + C4
# shard legs of bench.py, interleaved runs per setting of an environment
# variable. Usage: bash tools/enrich_ab.sh VAR "v1 v2" [rounds]
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/enrich_ab
mkdir -p $O
VAR=$1
VALS=$2
N=${3:-2}
for r in $(seq 1 $N); do
  for v in $VALS; do
    n=$(basename "$v")
    env $VAR=$v timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-rows --no-tick --no-breadth --steps 20 --warmup 3 \
      > $O/${VAR}_${n}_$r.json 2> $O/${VAR}_${n}_$r.err || { echo "bench $VAR=$v failed"; tail -5 $O/${VAR}_${n}_$r.err; exit 1; }
    python -c "import json; d=json.load(open('$O/${VAR}_${n}_$r.json')); print('$VAR=$n', 'headline', round(d['roofline']['kernel_ms'],3), round(d['roofline']['frac'],4), 'shard', round(d['shard']['kernel_ms'],3), round(d['shard']['frac'],4))"
  done
done
