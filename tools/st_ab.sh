# supertrend A/B: parity (tests/test_supertrend_gpu.py) per library, then
# tools/st_sweep.py-style timing of bq_supertrend_hlc at 12.5k x 2k
set -o pipefail
cd $GRAFT_REPO_ROOT
for lib in binquant_amd/lib/libbinquant_amd.so "$@"; do
  BQ_LIB_PATH=$PWD/$lib timeout -k 10 300 python -m pytest -x -q tests/test_supertrend_gpu.py -m gpu > gpurun_out/ab_test.log 2>&1 || { echo "TESTFAIL $lib"; tail -20 gpurun_out/ab_test.log; exit 1; }
  echo "parity ok $lib"
done
for rep in 1 2; do
  for lib in binquant_amd/lib/libbinquant_amd.so "$@"; do
    BQ_LIB_PATH=$PWD/$lib timeout -k 10 120 python - <<PY || exit 1
import torch, sys
sys.path.insert(0, '.')
from binquant_amd import engine
from binquant_amd.synth import device_panel
p = device_panel(12500, 2000, seed=1)
for _ in range(3): engine.supertrend(p['high'], p['low'], p['close'], period=10, multiplier=3.0)
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(10): engine.supertrend(p['high'], p['low'], p['close'], period=10, multiplier=3.0)
e1.record(); e1.synchronize()
print('$lib', round(e0.elapsed_time(e1) / 10, 4))
PY
  done
done
