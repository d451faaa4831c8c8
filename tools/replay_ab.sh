# A/B of the two replay kernels (tools/replay_ab.py), one process each
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
for impl in ring restage; do
  BQ_REPLAY_IMPL=$impl timeout -k 10 300 python3 $R/tools/replay_ab.py > $R/gpurun_out/replay_ab_$impl.jsonl || { echo "replay_ab $impl failed"; exit 1; }
done
echo REPLAY_AB_DONE
