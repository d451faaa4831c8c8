# A/B of environment settings on rows: bash tools/ab_env.sh "<rows>" "<VAR=val ...>" "<VAR=val ...>" ...
# -> gpurun_out/abe.log (each setting, each row, twice, interleaved)
set -e
mkdir -p gpurun_out
ROWS=$1; shift
for i in 1 2; do
  for setting in "$@"; do
    for row in $ROWS; do
      (export $setting; timeout -k 10 120 python -u tools/row_prof.py $row 2>/dev/null | sed "s/^/[$setting] /") >> gpurun_out/abe.log
    done
  done
done
