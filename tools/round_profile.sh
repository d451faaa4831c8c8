# Full round measurement on the GPU box: parity tests, smoke, bench line,
# rocprofv3 kernel trace + stats of the same bench, PMC passes.
# Usage: bash tools/round_profile.sh <tag>
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
TAG=${1:-r1}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
timeout -k 10 600 python -m pytest tests -m gpu -q > $O/gpu_tests.log 2>&1 || { echo GPU_TESTS_FAILED; tail -30 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo SMOKE_FAILED; tail $O/smoke.log; exit 1; }
timeout -k 10 600 python bench.py > $O/bench.json 2> $O/bench.err || { echo BENCH_FAILED; tail $O/bench.err; exit 1; }
cat $O/bench.json
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 $R/bench.py --no-cpu-baseline --no-rows --ticks 200 --store-ticks 10 > $O/trace_bench.json 2> $O/trace.err || { echo TRACE_FAILED; tail $O/trace.err; exit 1; }
rm -f $O/trace/run_kernel_trace.csv   # per-dispatch rows: large; the stats summary is what is kept
cd $R
bash tools/pmc_profile.sh gpurun_out/$TAG/pmc || exit 1
python tools/pmc_summary.py $O/pmc enrich_kernel $O/pmc_traffic.json $TAG > /dev/null
echo ROUND_PROFILE_DONE
