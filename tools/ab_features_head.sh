# A/B the features kernel at the headline shape through the bench's breadth
# leg (bq_market_features + bq_breadth_partial, 100k x 10k unless
# BQ_AB_SYMBOLS), parity first. Usage: bash tools/ab_features_head.sh lib.so ...
set -o pipefail
cd $GRAFT_REPO_ROOT
S=${BQ_AB_SYMBOLS:-100000}
for lib in binquant_amd/lib/libbinquant_amd.so "$@"; do
  BQ_LIB_PATH=$PWD/$lib timeout -k 10 300 python -m pytest tests/test_market_gpu.py -x -q > gpurun_out/ab_test.log 2>&1 || { echo "TESTFAIL $lib"; tail -20 gpurun_out/ab_test.log; exit 1; }
  echo "parity ok $lib"
done
for rep in 1 2; do
  for lib in binquant_amd/lib/libbinquant_amd.so "$@"; do
    BQ_LIB_PATH=$PWD/$lib timeout -k 10 300 python bench.py --symbols $S --no-shard --no-cpu-baseline --no-tick --no-rows --steps 2 --warmup 1 --breadth-steps 3 | python -c "import json,sys; d=json.load(sys.stdin); b=d['breadth']; print('$lib', $S, round(b['ms_per_step'],4))" || exit 1
  done
done
