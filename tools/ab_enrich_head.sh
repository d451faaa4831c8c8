# A/B the enrich kernel at the headline shape: parity (tests/test_enrich_gpu.py)
# on each library, then the headline leg (100k x 10k unless BQ_AB_SYMBOLS is
# set) per library, interleaved twice; prints kernel ms and the fraction of
# 8 TB/s. Usage: bash tools/ab_enrich_head.sh lib1.so lib2.so ...
set -o pipefail
cd $GRAFT_REPO_ROOT
S=${BQ_AB_SYMBOLS:-100000}
for lib in binquant_amd/lib/libbinquant_amd.so "$@"; do
  BQ_LIB_PATH=$PWD/$lib timeout -k 10 300 python -m pytest tests/test_enrich_gpu.py -x -q > gpurun_out/ab_test.log 2>&1 || { echo "TESTFAIL $lib"; tail -20 gpurun_out/ab_test.log; exit 1; }
  echo "parity ok $lib"
done
for rep in 1 2; do
  for lib in binquant_amd/lib/libbinquant_amd.so "$@"; do
    BQ_LIB_PATH=$PWD/$lib timeout -k 10 300 python bench.py --symbols $S --no-shard --no-cpu-baseline --no-tick --no-breadth --no-rows --steps 10 --warmup 2 | python -c "import json,sys; d=json.load(sys.stdin); r=d['roofline']; print('$lib', $S, round(r['kernel_ms'],4), round(r['frac'],4))" || exit 1
  done
done
