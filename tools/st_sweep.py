"""engine.supertrend time vs symbol count (latency- vs bandwidth-bound check)."""
import os
import sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from binquant_amd import engine
from binquant_amd.synth import device_panel

T = int(os.environ.get("ST_T", "2000"))
p = device_panel(16384, T, seed=99)
for S in [int(v) for v in sys.argv[1:]] or [1024, 4096, 8192, 12500, 16384]:
    h, l, c = p["high"][:S], p["low"][:S], p["close"][:S]
    engine.supertrend(h, l, c, exact=False)
    torch.cuda.synchronize()
    a, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(5):
        engine.supertrend(h, l, c, exact=False)
    e.record()
    torch.cuda.synchronize()
    print(f"S={S} ms={a.elapsed_time(e) / 5:.4f}")
