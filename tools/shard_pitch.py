"""Enrich kernel time at the C4 shard (12 500 x 10 000) against the output row
pitch (T + pad doubles): does the shard's gap to the headline follow the
address pattern of its concurrent row streams? (tools/shard_pmc.sh: the
shard's DRAM write credit stalls per candle are 8x the headline's.)
Interleaved rounds; HIP-event time per launch.
Usage: python tools/shard_pitch.py [S] [pad ...]"""
import sys

import torch

from binquant_amd import engine
from binquant_amd.engine import ENRICH_COLUMNS
from binquant_amd.synth import device_panel

T = 10_000
S = int(sys.argv[1]) if len(sys.argv) > 1 else 12_500
pads = [int(x) for x in sys.argv[2:]] or [0, 64]
p = device_panel(S, T, seed=1)
res = {pad: [] for pad in pads}
for rnd in range(3):
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
        res[pad].append(ev[0].elapsed_time(ev[1]) / 10)
        del bufs, out
for pad in pads:
    ms = min(res[pad])
    print(f"S {S} pad {pad:4d} ({(T + pad) * 8} B pitch): {' '.join(f'{x:.3f}' for x in res[pad])} ms, best "
          f"{S * T * 152 / (ms * 1e-3) / 8e12:.3f} of 8 TB/s", flush=True)
