set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out/d1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/d1/gpu_tests.log 2>&1 || { echo TESTS_FAILED; tail -30 gpurun_out/d1/gpu_tests.log; exit 1; }
tail -2 gpurun_out/d1/gpu_tests.log
timeout -k 10 300 python tools/row_costs.py > gpurun_out/d1/row_costs.log 2>&1 || { echo ROWS_FAILED; tail gpurun_out/d1/row_costs.log; exit 1; }
cp gpurun_out/row_costs.json gpurun_out/d1/
PIPES="zscore wilder_rsi adx failed_spike" bash tools/pipeline_profile.sh
