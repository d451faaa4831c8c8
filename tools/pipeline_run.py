"""Run one strategy pipeline a few times (for rocprofv3 kernel breakdowns).
Usage: python tools/pipeline_run.py <activity_burst|pump_score|failed_spike|top_gainer|adx|zscore|wilder_rsi> [S] [T]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from binquant_amd import signals, strategies
from binquant_amd.synth import device_panel

name = sys.argv[1]
S = int(sys.argv[2]) if len(sys.argv) > 2 else 12_500
T = int(sys.argv[3]) if len(sys.argv) > 3 else 2_000
p = device_panel(S, T, seed=3)
o, h, l, c, v = (p[k] for k in ("open", "high", "low", "close", "volume"))
qv = v * c
fn = {
    "activity_burst": lambda: strategies.activity_burst_features(o, h, l, c, v, qv),
    "pump_score": lambda: strategies.pump_score_features(o, h, l, c, v, c[0].clone()),
    "failed_spike": lambda: strategies.failed_spike_features(o, h, l, c, v, qv),
    "top_gainer": lambda: signals.top_gainer_features(o, h, l, c, v, qv),
    "adx": lambda: signals.adx(h, l, c),
    "zscore": lambda: signals.zscore(c),
    "wilder_rsi": lambda: signals.wilder_rsi(c),
}[name]
for _ in range(3):
    fn()
torch.cuda.synchronize()
