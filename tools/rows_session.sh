set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/s1
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_enrich_gpu.py tests/test_signals_gpu.py tests/test_market_gpu.py tests/test_beta_corr.py tests/test_panel_fixtures_gpu.py -m gpu > gpurun_out/s1/tests.log 2>&1 || { echo TESTS_FAILED; tail -30 gpurun_out/s1/tests.log; exit 1; }
tail -1 gpurun_out/s1/tests.log
timeout -k 10 600 python -u bench.py --no-cpu-baseline --no-tick > gpurun_out/s1/bench.json 2> gpurun_out/s1/bench.err || { echo BENCH_FAILED; tail gpurun_out/s1/bench.err; exit 1; }
python - <<'PY'
import json
d=json.load(open('gpurun_out/s1/bench.json'))
print('headline', round(d['ms_per_step'],3), round(d['roofline']['frac'],4), 'shard', round(d['shard']['kernel_ms'],3), round(d['shard']['frac'],4), 'breadth', round(d['breadth']['ms_per_step'],3))
for k,v in d['rows'].items():
    if isinstance(v, dict) and 'ms' in v: print(k, round(v['ms'],4), round(v['frac'],4))
PY
