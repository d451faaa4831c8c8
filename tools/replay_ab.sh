# A/B of the replay kernels (tools/replay_ab.py), one process each: LDS ring,
# per-class re-staged and mixed-class re-staged at each symbols-per-wave
# setting, and the automatic choice. Digests must agree across all lines.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/replay_ab
cd $R
run() {   # tag, env...
  local tag=$1; shift
  env "$@" timeout -k 10 300 python3 tools/replay_ab.py > gpurun_out/replay_ab/$tag.jsonl || { echo "replay_ab $tag failed"; exit 1; }
}
run auto BQ_X=0
[ -n "$QUICK" ] || run ring BQ_REPLAY_IMPL=ring
for spw in ${SPWS:-64 32 16 8}; do
  run restage$spw BQ_REPLAY_IMPL=restage BQ_REPLAY_SPW=$spw
  run mixed$spw BQ_REPLAY_IMPL=mixed BQ_REPLAY_SPW=$spw
done
echo REPLAY_AB_DONE
