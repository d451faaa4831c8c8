# The C4 shard against the headline: enrich at 12 288 symbols (16 whole rounds
# of 768 resident workgroups), 12 500 (16.3), 13 056 (17) per GPU and the 100k
# headline, for the in-tree library and variants (tools/build_variant.sh):
# bash tools/shard_tail.sh [variant ...] -> gpurun_out/shard_tail.log
set -e
A="--no-cpu-baseline --no-rows --no-tick --no-breadth --no-shard --steps 10 --warmup 2"
for v in base "$@"; do
  if [ "$v" = base ]; then unset BQ_LIB_PATH; else export BQ_LIB_PATH=binquant_amd/lib/variants/lib_$v.so; fi
  for s in 12288 12500 100000; do
    timeout -k 10 300 python -u bench.py $A --symbols $s 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('$v', $s, round(d['roofline']['kernel_ms'],4), round(d['roofline']['frac'],4))" >> gpurun_out/shard_tail.log
  done
done
