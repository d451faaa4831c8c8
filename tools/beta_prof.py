"""Time engine.beta_corr at 12.5k x 2k (run under rocprofv3 --kernel-trace --stats)."""
import sys
sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__))))
import torch
from binquant_amd import engine
from binquant_amd.synth import device_panel

p = device_panel(12500, 2000, seed=99)
c = p["close"]
b = c[0].clone()
engine.beta_corr(c, b, 50)
torch.cuda.synchronize()
a, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
a.record()
for _ in range(10):
    engine.beta_corr(c, b, 50)
e.record()
torch.cuda.synchronize()
print("beta_corr ms", a.elapsed_time(e) / 10)
