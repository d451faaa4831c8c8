# Kernel-time A/B of library variants on one row under rocprofv3 (the
# variants from tools/build_variant.sh): bash tools/ab_kernel.sh <row> <kernel-substring> v1 v2 ...
# -> gpurun_out/abk_<row>.log: per variant the kernel's average duration (base = in-tree library)
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
ROW=$1; KSUB=$2; shift 2
for v in base "$@"; do
  if [ "$v" = base ]; then unset BQ_LIB_PATH; else export BQ_LIB_PATH=binquant_amd/lib/variants/lib_$v.so; fi
  rm -rf gpurun_out/abk_$v
  timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/abk_$v -o run -- python3 tools/row_prof.py $ROW > gpurun_out/abk_$v.log 2>&1
  f=$(find gpurun_out/abk_$v -name "*kernel_stats.csv" | head -1)
  python3 - "$f" "$KSUB" "$v" "$(grep ms/call gpurun_out/abk_$v.log)" >> gpurun_out/abk_$ROW.log <<'PY'
import csv, sys
f, ks, v, row = sys.argv[1:5]
for r in csv.DictReader(open(f)):
    if ks in r["Name"]:
        print(f"{v} {float(r['AverageNs']) / 1e3:.1f} us x{r['Calls']} {r['Name'][:60]} | {row}")
PY
done
