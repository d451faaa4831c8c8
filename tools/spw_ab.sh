# replay symbols-per-wave: automatic choice vs forced 64, pipeline breakdowns
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -m pytest tests/test_rolling_impls_gpu.py tests/test_strategies_gpu.py tests/test_signals_gpu.py -q -x > gpurun_out/spw_tests.log 2>&1 || { tail -30 gpurun_out/spw_tests.log; exit 1; }
tail -n 1 gpurun_out/spw_tests.log
for p in ${PIPES:-adx zscore wilder_rsi top_gainer pump_score failed_spike}; do
  for mode in auto 64; do
    if [ $mode = 64 ]; then export BQ_REPLAY_SPW=64; else unset BQ_REPLAY_SPW; fi
    (cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/pipe_${mode}_$p -o run -- python3 $GRAFT_REPO_ROOT/tools/pipeline_run.py $p > /dev/null 2>&1) || { echo "prof $mode $p failed"; exit 1; }
  done
done
echo SPW_AB_DONE
