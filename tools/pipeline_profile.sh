# rocprofv3 kernel breakdown of each strategy pipeline (tools/pipeline_run.py)
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd /tmp
for p in ${PIPES:-activity_burst pump_score failed_spike top_gainer adx zscore wilder_rsi}; do
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/pipe${PT:-}_$p -o run -- python3 $R/tools/pipeline_run.py $p ${PS:-12500} ${PT:-2000} > /dev/null 2>&1 || { echo "prof $p failed"; exit 1; }
done
echo PIPE_DONE
