"""Enrich kernel time at the C4 shard (12 500 x 10 000) with the output rows
padded (row pitch T + pad) and at 100k for reference: does the shard's gap
to the headline follow the address pattern of its concurrent row streams?
Usage: python tools/shard_pitch.py"""
import torch

from binquant_amd import engine
from binquant_amd.engine import ENRICH_COLUMNS
from binquant_amd.synth import device_panel

T = 10_000
for S, pads in ((12_500, (0, 64)), (100_000, (0, 64))):
    p = device_panel(S, T, seed=1)
    for pad in pads:
        bufs = {k: torch.empty((S, T + pad), dtype=torch.float64, device="cuda") for k in ENRICH_COLUMNS}
        out = {k: v[:, :T] for k, v in bufs.items()}
        f = lambda: engine.enrich(p["open"], p["high"], p["low"], p["close"], p["volume"], out=out)  # noqa: E731
        for _ in range(2):
            f()
        torch.cuda.synchronize()
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
        ev[0].record()
        for _ in range(10):
            f()
        ev[1].record()
        torch.cuda.synchronize()
        ms = ev[0].elapsed_time(ev[1]) / 10
        print(f"S {S} pad {pad}: {ms:.3f} ms, {S * T * 152 / (ms * 1e-3) / 8e12:.3f} of 8 TB/s", flush=True)
        del bufs, out
    del p
    torch.cuda.empty_cache()
