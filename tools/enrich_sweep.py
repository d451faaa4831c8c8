"""Enrich kernel time vs panel rows (tail / occupancy diagnosis): HIP-event
mean over reps, per-symbol ns and fraction of 8 TB/s.
Usage: python tools/enrich_sweep.py S1 S2 ... [--T 10000]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from binquant_amd import engine
from binquant_amd._lib import ENRICH_COLUMNS
from binquant_amd.synth import device_panel

args = [a for a in sys.argv[1:] if not a.startswith("--")]
T = 10_000
for S in map(int, args):
    p = device_panel(S, T, seed=1)
    out = {k: torch.empty((S, T), dtype=torch.float64, device="cuda") for k in ENRICH_COLUMNS}
    f = lambda: engine.enrich(p["open"], p["high"], p["low"], p["close"], p["volume"], out=out)  # noqa: E731
    for _ in range(3):
        f()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    reps = max(3, int(200_000 / S))
    a.record()
    for _ in range(reps):
        f()
    b.record()
    torch.cuda.synchronize()
    ms = a.elapsed_time(b) / reps
    print(f"S={S} ms={ms:.4f} ns/symbol={ms * 1e6 / S:.1f} frac={S * T * 152 / (ms * 1e-3) / 8e12:.4f}", flush=True)
    del p, out
    torch.cuda.empty_cache()
