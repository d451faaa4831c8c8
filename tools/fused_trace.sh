cd $GRAFT_REPO_ROOT
for p in activity_burst pump_score failed_spike top_gainer; do echo "== $p"; BQ_FUSED_TRACE=1 timeout -k 10 60 python tools/pipeline_run.py $p 100 2000 2>&1 | grep fused | head -8; done
