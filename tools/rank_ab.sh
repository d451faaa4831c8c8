# A/B of the two order-statistic kernels (tools/rank_ab.py), one process each
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
for impl in ${IMPLS:-lane tile stencil}; do
  BQ_RANK_IMPL=$impl timeout -k 10 300 python3 $R/tools/rank_ab.py > $R/gpurun_out/rank_ab_$impl.jsonl || { echo "rank_ab $impl failed"; exit 1; }
done
echo RANK_AB_DONE
