# parity of the rolling / strategy kernels, then the bench's rows leg only
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/rq
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread ${TESTS:-tests/test_rolling_impls_gpu.py tests/test_strategies_gpu.py tests/test_panel_fixtures_gpu.py tests/test_signals_gpu.py} -m gpu > gpurun_out/rq/tests.log 2>&1 || { echo TESTS_FAILED; tail -30 gpurun_out/rq/tests.log; exit 1; }
tail -1 gpurun_out/rq/tests.log
timeout -k 10 600 python -u bench.py --no-cpu-baseline --no-tick --no-shard --no-breadth --symbols 12500 --steps 3 --warmup 1 > gpurun_out/rq/bench.json 2> gpurun_out/rq/bench.err || { echo BENCH_FAILED; tail gpurun_out/rq/bench.err; exit 1; }
python - <<'PY'
import json
d=json.load(open('gpurun_out/rq/bench.json'))
for k,v in d['rows'].items():
    if isinstance(v, dict) and 'ms' in v: print(k, round(v['ms'],4), round(v['frac'],4))
for k,v in d.get('live',{}).items():
    if isinstance(v, dict): print('live', k, v)
PY
