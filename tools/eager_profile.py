"""cProfile of one eager strategy pipeline call at the live shape (host-side
cost of building the fused programs and the rolling job tables).
Usage: python tools/eager_profile.py <pipeline> [S] [T]"""
import cProfile
import os
import pstats
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from binquant_amd import signals, strategies
from binquant_amd.synth import device_panel

name = sys.argv[1]
S = int(sys.argv[2]) if len(sys.argv) > 2 else 1000
T = int(sys.argv[3]) if len(sys.argv) > 3 else 400
p = device_panel(S, T, seed=3)
o, h, l, c, v = (p[k] for k in ("open", "high", "low", "close", "volume"))
qv = v * c
fn = {
    "activity_burst": lambda: strategies.activity_burst_features(o, h, l, c, v, qv),
    "pump_score": lambda: strategies.pump_score_features(o, h, l, c, v, c[0].clone()),
    "failed_spike": lambda: strategies.failed_spike_features(o, h, l, c, v, qv),
    "top_gainer": lambda: signals.top_gainer_features(o, h, l, c, v, qv),
}[name]
for _ in range(3):
    fn()
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(20):
    fn()
torch.cuda.synchronize()
print(f"{name}: eager {(time.perf_counter() - t0) / 20 * 1e3:.3f} ms per call")
pr = cProfile.Profile()
pr.enable()
for _ in range(20):
    fn()
torch.cuda.synchronize()
pr.disable()
pstats.Stats(pr).sort_stats("cumulative").print_stats(25)
