# Full round measurement on the GPU box: parity tests (recording the fused
# program manifest), smoke, the default bench line, rocprofv3 kernel trace +
# stats of the headline-only bench command (the enrich_kernel launches are all
# the 100k x 10k headline), PMC passes of the same command.
# Usage: bash tools/round_profile.sh <tag> [skip-tests]
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
TAG=${1:-r2}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
if [ -z "$2" ]; then
  BQ_FUSED_MANIFEST=$O/manifest_tests.jsonl timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo GPU_TESTS_FAILED; grep -E "Error|assert|FAILED" $O/gpu_tests.log | head -30; tail -3 $O/gpu_tests.log; exit 1; }
  tail -1 $O/gpu_tests.log
fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo SMOKE_FAILED; tail $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 900 python -u bench.py > $O/bench.json 2> $O/bench.err || { echo BENCH_FAILED; tail $O/bench.err; exit 1; }
python -c "import json; d=json.load(open('$O/bench.json')); print(d['value'], d['ms_per_step'], d['roofline']['frac'], d['shard']['frac'], d['store']['p99_ms'], d['tick']['p99_ms'], d['cpu_baseline']['value'])"
HEAD="--no-cpu-baseline --no-rows --no-tick --no-shard --no-breadth --steps 20 --warmup 5"
cd /tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 $R/bench.py $HEAD > $O/trace_bench.json 2> $O/trace.err || { echo TRACE_FAILED; tail $O/trace.err; exit 1; }
cd $R
python tools/trace_summary.py $O/trace enrich_kernel > $O/trace_summary.txt && cat $O/trace_summary.txt
rm -f $O/trace/run_kernel_trace.csv
bash tools/pmc_profile.sh gpurun_out/$TAG/pmc || exit 1
python tools/pmc_summary.py $O/pmc enrich_kernel $O/pmc_traffic.json $TAG 1000000000 > /dev/null
python -c "import json; d=json.load(open('$O/pmc_traffic.json'))['enrich_kernel']; print('traffic/launch', d['bytes_per_launch'], 'LDS conflicts', d['counters_mean_per_dispatch'].get('SQ_LDS_BANK_CONFLICT'))"
echo ROUND_PROFILE_DONE
