"""Enrich kernel time vs row pitch (ld) of inputs and outputs at S x T
(HBM channel / page locality diagnosis). Usage: python tools/enrich_ld_sweep.py S T ld1 ld2 ..."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from binquant_amd import engine
from binquant_amd._lib import ENRICH_COLUMNS
from binquant_amd.synth import device_panel

S, T = int(sys.argv[1]), int(sys.argv[2])
src = device_panel(S, T, seed=1)
for ld in map(int, sys.argv[3:]):
    p = {}
    for k, v in src.items():
        buf = torch.empty((S, ld), dtype=torch.float64, device="cuda")
        buf[:, :T].copy_(v)
        p[k] = buf[:, :T]
    ob = {k: torch.empty((S, ld), dtype=torch.float64, device="cuda") for k in ENRICH_COLUMNS}
    out = {k: v[:, :T] for k, v in ob.items()}
    f = lambda: engine.enrich(p["open"], p["high"], p["low"], p["close"], p["volume"], out=out)  # noqa: E731
    for _ in range(3):
        f()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(20):
        f()
    b.record()
    torch.cuda.synchronize()
    ms = a.elapsed_time(b) / 20
    print(f"ld={ld} ms={ms:.4f} frac={S * T * 152 / (ms * 1e-3) / 8e12:.4f}", flush=True)
    del p, ob, out
    torch.cuda.empty_cache()
