# market-features parity tests, then the C5 breadth leg (features + partials) twice
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/quick
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread -k "market or breadth or distributed or regime" > gpurun_out/quick/gpu_tests.log 2>&1 || { echo GPU_TESTS_FAILED; tail -40 gpurun_out/quick/gpu_tests.log; exit 1; }
tail -1 gpurun_out/quick/gpu_tests.log
for i in 1 2; do
  timeout -k 10 120 python bench.py --no-rows --no-tick --no-cpu-baseline --steps 10 > gpurun_out/quick/b$i.json 2>/dev/null || exit 1
  python -c "import json;d=json.load(open('gpurun_out/quick/b$i.json'));print('enrich', round(d['roofline']['kernel_ms'],3), 'breadth leg ms', round(d['breadth']['ms_per_step'],3))"
done
cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/quick/prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --no-rows --no-tick --no-cpu-baseline --steps 5 > /dev/null 2>&1 || exit 1
grep -E "features_kernel|breadth_kernel" $GRAFT_REPO_ROOT/gpurun_out/quick/prof/run_kernel_stats.csv | cut -c1-120
