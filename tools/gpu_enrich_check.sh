set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 300 python -m pytest tests/test_enrich_gpu.py -x -q > gpurun_out/t_enrich.log 2>&1 || { echo TESTFAIL; tail -30 gpurun_out/t_enrich.log; exit 1; }
tail -2 gpurun_out/t_enrich.log
timeout -k 10 300 python bench.py --no-cpu-baseline --no-tick --no-breadth > gpurun_out/bench.json 2> gpurun_out/bench.err || { echo BENCHFAIL; tail gpurun_out/bench.err; exit 1; }
cat gpurun_out/bench.json
