set -o pipefail
cd $GRAFT_REPO_ROOT
for lib in ${LIBS:-binquant_amd/lib/libbinquant_amd.so}; do
BQ_LIB_PATH=$PWD/$lib timeout -k 10 300 python -c "
import sys, json; sys.path.insert(0,'.'); import torch
from binquant_amd import engine
from binquant_amd.synth import device_panel
p = device_panel(12500, 2000, seed=99); c = p['close']; b = c[0].clone()
engine.beta_corr(c, b, 50); torch.cuda.synchronize()
a, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
a.record()
for _ in range(10): engine.beta_corr(c, b, 50)
e.record(); torch.cuda.synchronize(); print('$lib', a.elapsed_time(e)/10)
" || exit 1
done
