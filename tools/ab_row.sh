# A/B of library variants on one row (tools/build_variant.sh builds them):
# bash tools/ab_row.sh <row> v1 v2 ... -> gpurun_out/ab_<row>.log (base = the in-tree library)
set -e
mkdir -p gpurun_out
ROW=$1; shift
for i in 1 2; do
  for v in base "$@"; do
    if [ "$v" = base ]; then timeout -k 10 120 python -u tools/row_prof.py $ROW 2>/dev/null | sed 's/^/base /' >> gpurun_out/ab_$ROW.log
    else BQ_LIB_PATH=binquant_amd/lib/variants/lib_$v.so timeout -k 10 120 python -u tools/row_prof.py $ROW 2>/dev/null | sed "s/^/$v /" >> gpurun_out/ab_$ROW.log; fi
  done
done
