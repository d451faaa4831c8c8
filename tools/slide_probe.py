"""One order-statistic job on a NaN-free 12.5k x 2k synthetic panel (the
strategy rows' shape), repeated: the program rocprofv3 traces / counts to
compare the slide and tile rank kernels (BQ_RANK_IMPL=slide|tile).

    python tools/slide_probe.py <window> <median|quantile|qlower> <q> <min_periods> <shift> [reps]
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from binquant_amd import engine  # noqa: E402
from binquant_amd.synth import device_panel  # noqa: E402

w, stat, q, mp, sh = int(sys.argv[1]), sys.argv[2], float(sys.argv[3]), int(sys.argv[4]), int(sys.argv[5])
reps = int(sys.argv[6]) if len(sys.argv) > 6 else 10
x = device_panel(12_500, 2_000, seed=5)["volume"].clone()
out = engine.rolling(x, w, stat, q=q, min_periods=mp, shift=sh)
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(reps):
    engine.rolling(x, w, stat, q=q, min_periods=mp, shift=sh, out=out)
e1.record()
torch.cuda.synchronize()
print(os.environ.get("BQ_RANK_IMPL", "auto"), w, stat, q, "ms", round(e0.elapsed_time(e1) / reps, 4), flush=True)
