# rank kernels: parity tests with the default library, then tools/rank_ab.py
# per implementation for the default and a variant library (BQ_AB_LIB)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/rk
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_rolling_impls_gpu.py tests/test_strategies_gpu.py tests/test_panel_fixtures_gpu.py -m gpu > gpurun_out/rk/tests.log 2>&1 || { echo TESTS_FAILED; tail -30 gpurun_out/rk/tests.log; exit 1; }
tail -1 gpurun_out/rk/tests.log
for impl in tile stencil; do
  BQ_RANK_IMPL=$impl timeout -k 10 300 python3 tools/rank_ab.py > gpurun_out/rk/new_$impl.jsonl || { echo "rank_ab $impl failed"; exit 1; }
  BQ_LIB_PATH=$PWD/$BQ_AB_LIB BQ_RANK_IMPL=$impl timeout -k 10 300 python3 tools/rank_ab.py > gpurun_out/rk/old_$impl.jsonl || { echo "rank_ab old $impl failed"; exit 1; }
done
echo RANK_SESSION_DONE
