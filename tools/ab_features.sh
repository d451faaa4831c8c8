# A/B of the market-features kernel: parity tests then the breadth leg timing.
set -o pipefail
cd $GRAFT_REPO_ROOT
for lib in binquant_amd/lib/libbinquant_amd.so "$@"; do
  echo "== $lib"
  BQ_LIB_PATH=$PWD/$lib timeout -k 10 300 python -m pytest tests/test_market_gpu.py tests/test_store_gpu.py -x -q > gpurun_out/ab_test.log 2>&1 || { echo TESTFAIL; tail -20 gpurun_out/ab_test.log; exit 1; }
  for i in 1 2; do
    BQ_LIB_PATH=$PWD/$lib timeout -k 10 300 python bench.py --no-cpu-baseline --no-tick --no-rows --steps 3 --breadth-steps 10 | python -c "import json,sys; d=json.load(sys.stdin); print(round(d['breadth']['ms_per_step'],4))" || exit 1
  done
done
