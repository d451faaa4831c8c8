"""Enrich kernel time at the C4 shard against the relative placement of the 14
output columns: each column its own allocation (as engine.enrich_outputs;
the caching allocator puts them on 2 MiB boundaries, so the 14 streams a
workgroup writes at one (row, t) share their low address bits), or all 14 in
ONE buffer with column c starting c * (column bytes + stagger) in. Row pitch
T + 192 doubles throughout. Interleaved rounds; HIP-event time per launch.
Usage: PYTHONPATH=. python tools/shard_stagger.py [S] [stagger_bytes ...]
(stagger -1 = separate allocations)"""
import sys

import torch

from binquant_amd import engine
from binquant_amd.engine import ENRICH_COLUMNS, ENRICH_ROW_PAD
from binquant_amd.synth import device_panel

T = 10_000
S = int(sys.argv[1]) if len(sys.argv) > 1 else 12_500
stags = [int(x) for x in sys.argv[2:]] or [-1, 0, 256, 4096]
P = T + ENRICH_ROW_PAD
p = device_panel(S, T, seed=1)
res = {s: [] for s in stags}


def outputs(stag):
    if stag < 0:
        return None, {k: torch.empty((S, P), dtype=torch.float64, device="cuda")[:, :T] for k in ENRICH_COLUMNS}
    col = S * P * 8 + stag                    # bytes per column slot
    assert col % 16 == 0
    n = len(ENRICH_COLUMNS)
    buf = torch.empty(n * col // 8, dtype=torch.float64, device="cuda")
    out = {}
    for c, k in enumerate(ENRICH_COLUMNS):
        out[k] = buf[c * col // 8: c * col // 8 + S * P].view(S, P)[:, :T]
    return buf, out


for rnd in range(3):
    for stag in stags:
        buf, out = outputs(stag)
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
        res[stag].append(ev[0].elapsed_time(ev[1]) / 10)
        del buf, out
        torch.cuda.empty_cache()
for stag in stags:
    ms = min(res[stag])
    name = "separate" if stag < 0 else f"one buffer, stagger {stag} B"
    print(f"S {S} {name:28s}: {' '.join(f'{x:.3f}' for x in res[stag])} ms, best "
          f"{S * T * 152 / (ms * 1e-3) / 8e12:.3f} of 8 TB/s", flush=True)
