# A/B the enrich kernel: parity on each variant, then the headline leg at
# 12.5k x 10k (kernel ms, frac), interleaved twice. Usage: bash tools/ab_enrich.sh lib1.so lib2.so ...
set -o pipefail
cd $GRAFT_REPO_ROOT
for lib in binquant_amd/lib/libbinquant_amd.so "$@"; do
  BQ_LIB_PATH=$PWD/$lib timeout -k 10 300 python -m pytest tests/test_enrich_gpu.py -x -q > gpurun_out/ab_test.log 2>&1 || { echo "TESTFAIL $lib"; tail -20 gpurun_out/ab_test.log; exit 1; }
done
for rep in 1 2; do
  for lib in binquant_amd/lib/libbinquant_amd.so "$@"; do
    BQ_LIB_PATH=$PWD/$lib timeout -k 10 300 python bench.py --symbols 12500 --no-shard --no-cpu-baseline --no-tick --no-breadth --no-rows --steps 30 | python -c "import json,sys; d=json.load(sys.stdin); r=d['roofline']; print('$lib', round(r['kernel_ms'],4), round(r['frac'],4))" || exit 1
  done
done
