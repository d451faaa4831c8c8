# A/B of order-statistic kernel variants (tools/build_variant.sh) on the
# strategies' windows: bash tools/ab_slide.sh v1 v2 ... -> gpurun_out/ab_slide.log
set -e
mkdir -p gpurun_out
for i in 1 2; do
  for v in base "$@"; do
    for args in "19 median 0.5 19 2" "48 quantile 0.8 48 1" "60 quantile 0.85 20 1" "80 quantile 0.92 20 1"; do
      if [ "$v" = base ]; then L=binquant_amd/lib/libbinquant_amd.so; else L=binquant_amd/lib/variants/lib_$v.so; fi
      BQ_LIB_PATH=$L timeout -k 10 120 python -u tools/slide_probe.py $args 2>/dev/null | sed "s/^/$v /" >> gpurun_out/ab_slide.log
    done
  done
done
