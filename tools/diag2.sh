set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out/d2
timeout -k 10 300 python -u -m pytest tests/test_strategies_gpu.py tests/test_signals_gpu.py tests/test_rolling_impls_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/d2/gpu_tests.log 2>&1 || { echo TESTS_FAILED; tail -30 gpurun_out/d2/gpu_tests.log; exit 1; }
tail -2 gpurun_out/d2/gpu_tests.log
bash tools/replay_ab.sh
timeout -k 10 300 python tools/row_costs.py > gpurun_out/d2/row_costs.log 2>&1 || { echo ROWS_FAILED; tail gpurun_out/d2/row_costs.log; exit 1; }
