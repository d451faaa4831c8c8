# rows leg (12.5k x 2k, HIP events) for the default library and variants,
# interleaved twice; parity of the rolling / strategy tests on each variant.
# Usage: bash tools/rows_ab.sh lib.so ...
set -o pipefail
cd $GRAFT_REPO_ROOT
for lib in binquant_amd/lib/libbinquant_amd.so "$@"; do
  BQ_LIB_PATH=$PWD/$lib timeout -k 10 300 python -m pytest -x -q tests/test_rolling_impls_gpu.py tests/test_strategies_gpu.py tests/test_panel_fixtures_gpu.py -m gpu > gpurun_out/ab_test.log 2>&1 || { echo "TESTFAIL $lib"; tail -20 gpurun_out/ab_test.log; exit 1; }
  echo "parity ok $lib"
done
for rep in 1 2; do
  for lib in binquant_amd/lib/libbinquant_amd.so "$@"; do
    BQ_LIB_PATH=$PWD/$lib timeout -k 10 300 python bench.py --no-cpu-baseline --no-tick --no-shard --no-breadth --symbols 12500 --steps 2 --warmup 1 | python -c "
import json,sys; d=json.load(sys.stdin)
print('$lib', ' '.join(f\"{k.split('_',1)[1] if '_' in k else k}={v['ms']:.3f}\" for k,v in d['rows'].items() if isinstance(v, dict) and 'ms' in v))" || exit 1
  done
done
