# A/B kernel variants on one box: parity tests on each variant, then bench.
set -o pipefail
cd $GRAFT_REPO_ROOT
for lib in binquant_amd/lib/libbinquant_amd.so "$@"; do
  echo "== $lib"
  BQ_LIB_PATH=$PWD/$lib timeout -k 10 300 python -m pytest tests/test_enrich_gpu.py -x -q > gpurun_out/ab_test.log 2>&1 || { echo TESTFAIL; tail -20 gpurun_out/ab_test.log; exit 1; }
  for i in 1 2; do
    BQ_LIB_PATH=$PWD/$lib timeout -k 10 300 python bench.py --no-cpu-baseline --no-tick --no-breadth --steps 30 | python -c "import json,sys; d=json.load(sys.stdin); print(round(d['ms_per_step'],4), round(d['roofline']['frac'],4))" || exit 1
  done
done
