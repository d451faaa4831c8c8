# pipeline breakdown for the default library and each variant library given ($@)
set -o pipefail
cd $GRAFT_REPO_ROOT
for lib in binquant_amd/lib/libbinquant_amd.so "$@"; do
  tag=$(basename $lib .so)
  for p in ${PIPES:-failed_spike adx wilder_rsi}; do
    (cd /tmp && BQ_LIB_PATH=$GRAFT_REPO_ROOT/$lib timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/pipe_${tag}_$p -o run -- python3 $GRAFT_REPO_ROOT/tools/pipeline_run.py $p > /dev/null 2>&1) || { echo "prof $tag $p failed"; exit 1; }
  done
done
echo PIPE_AB_DONE
