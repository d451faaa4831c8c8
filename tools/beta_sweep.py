"""engine.beta_corr time vs symbol count at T=2000 (wave-quantisation check)."""
import os
import sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from binquant_amd import engine
from binquant_amd.synth import device_panel

p = device_panel(16384, 2000, seed=99)
c = p["close"]
b = c[0].clone()
for S in [int(v) for v in sys.argv[1:]] or [3072, 6144, 9216, 12288, 12500, 13000, 15360, 16384]:
    cs = c[:S]
    engine.beta_corr(cs, b, 50)
    torch.cuda.synchronize()
    a, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(10):
        engine.beta_corr(cs, b, 50)
    e.record()
    torch.cuda.synchronize()
    ms = a.elapsed_time(e) / 10
    print(f"S={S} ms={ms:.4f} us_per_1k={1000 * ms / S * 1000:.2f}")
