"""Run one engine entry point a few times at 12.5k x 2k (for rocprofv3 kernel
breakdowns): python tools/call_prof.py supertrend|beta_corr|join_returns|market_features"""
import os
import sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from binquant_amd import engine
from binquant_amd.synth import device_panel

name = sys.argv[1]
S, T = (int(sys.argv[2]), int(sys.argv[3])) if len(sys.argv) > 3 else (12500, 2000)
p = device_panel(S, T, seed=99)
h, l, c = p["high"], p["low"], p["close"]
ts = (1_700_000_000_000 + 900_000 * torch.arange(T, device=c.device, dtype=torch.int64)).expand(S, T).contiguous()
calls = {
    "join_returns": lambda: engine.join_returns(ts, c, ts[0], c[0].clone()),
    "supertrend": lambda: engine.supertrend(h, l, c, period=10, multiplier=3.0),
    "beta_corr": lambda: engine.beta_corr(c, c[0].clone(), 50),
    "market_features": lambda: engine.market_features(h, l, c, max_bars=400),
}
fn = calls[name]
for _ in range(2):
    fn()
torch.cuda.synchronize()
a, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
a.record()
for _ in range(5):
    fn()
e.record()
torch.cuda.synchronize()
print(name, "ms", a.elapsed_time(e) / 5)
