# Timing only (no parity): the headline leg at 12.5k x 10k per library, interleaved twice.
set -o pipefail
cd $GRAFT_REPO_ROOT
for rep in 1 2; do
  for lib in binquant_amd/lib/libbinquant_amd.so "$@"; do
    BQ_LIB_PATH=$PWD/$lib timeout -k 10 300 python bench.py --symbols 12500 --no-shard --no-cpu-baseline --no-tick --no-breadth --no-rows --steps 30 | python -c "import json,sys; d=json.load(sys.stdin); r=d['roofline']; print('$lib', round(r['kernel_ms'],4), round(r['frac'],4))" || exit 1
  done
done
