"""Order-statistic kernels A/B (lane-sorted window vs wave-sorted tile union).
Run once per implementation: BQ_RANK_IMPL=lane|tile python tools/rank_ab.py
Prints one JSON line per (shape, job): mean ms over reps and a digest of the
output bytes (the two implementations must print identical digests)."""
import hashlib
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from binquant_amd import engine
from binquant_amd.synth import device_panel

# the pipelines' order-statistic jobs (window, stat, q, min_periods, shift)
JOBS = [(19, "median", 0.5, 19, 2), (80, "quantile", 0.92, 20, 1), (48, "quantile", 0.80, 48, 1),
        (60, "quantile", 0.85, 20, 1), (3, "max", 1.0, 1, 1), (6, "max", 1.0, 6, 1), (6, "min", 0.0, 6, 1),
        (96, "median", 0.5, 1, 0), (24, "quantile", 0.3, 5, 0), (96, "qlower", 0.8, 20, 0)]
impl = os.environ.get("BQ_RANK_IMPL", "auto")
for S, T, reps in ((1000, 400, 50), (12_500, 2_000, 10)):
    p = device_panel(S, T, seed=5)
    x = p["volume"].clone()
    x[:, 7::97] = float("nan")   # NaN gaps
    x[3, 100:160] = 1.0          # a constant run
    for w, stat, q, mp, sh in JOBS:
        out = engine.rolling(x, w, stat, q=q, min_periods=mp, shift=sh)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            engine.rolling(x, w, stat, q=q, min_periods=mp, shift=sh, out=out)
        e1.record()
        torch.cuda.synchronize()
        dig = hashlib.sha1(out.cpu().numpy().tobytes()).hexdigest()[:16]
        print(json.dumps({"impl": impl, "S": S, "T": T, "w": w, "stat": stat, "q": q,
                          "ms": e0.elapsed_time(e1) / reps, "digest": dig}), flush=True)
