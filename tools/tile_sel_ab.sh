# A/B of the 128-output tile rank kernels (bit selection vs the walk) on the
# rows that use windows > 65: leadership (w 96, q 0.8) and activity burst (w 80, q 0.92).
set -o pipefail
cd $GRAFT_REPO_ROOT
for sel in 1 0 1 0; do
  for row in a20_leadership a17_activity_burst; do
    BQ_TILE_SEL=$sel timeout -k 10 120 python tools/row_prof.py $row | sed "s/^/sel=$sel /" || exit 1
  done
done
