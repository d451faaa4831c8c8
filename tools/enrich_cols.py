"""Enrich kernel time per column subset at a given shape (HIP events on the
launch stream): which part of the per-tile work binds the kernel once the
memory pattern allows more? Usage: python tools/enrich_cols.py [S] [T]
(library from BQ_LIB_PATH as usual). One JSON line per subset."""

import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from binquant_amd import engine  # noqa: E402
from binquant_amd._lib import ENRICH_COLUMNS  # noqa: E402

S = int(sys.argv[1]) if len(sys.argv) > 1 else 100_000
T = int(sys.argv[2]) if len(sys.argv) > 2 else 10_000
dev = torch.device("cuda", 0)
g = torch.Generator(device=dev).manual_seed(0)
ins = []
for _ in range(5):
    x = torch.empty((S, T), dtype=torch.float64, device=dev)
    for a in range(0, S, 12_500):
        b = min(S, a + 12_500)
        r = torch.randn((b - a, T), dtype=torch.float64, device=dev, generator=g).mul_(0.002)
        x[a:b] = torch.cumsum(r, 1).exp_().mul_(100.0)
        del r
    ins.append(x)
o, h, l, c, v = ins
h.copy_(torch.maximum(o, c) * 1.001)
l.copy_(torch.minimum(o, c) * 0.999)
out = {k: torch.empty((S, T), dtype=torch.float64, device=dev) for k in ENRICH_COLUMNS}
subsets = {
    "all14": ENRICH_COLUMNS,
    "ema4": ("macd", "macd_signal", "ema20", "ema50"),
    "win10": tuple(k for k in ENRICH_COLUMNS if k not in ("macd", "macd_signal", "ema20", "ema50")),
    "ma3": ("ma_7", "ma_25", "ma_100"),
    "short5": ("rsi", "ATR", "twap", "mfi", "bb_upper"),
    "one": ("ma_7",),
}
st = torch.cuda.current_stream()
for name, cols in subsets.items():
    sub = {k: out[k] for k in cols}
    for _ in range(2):
        engine.enrich(o, h, l, c, v, columns=cols, out=sub)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    n = 5
    e0.record(st)
    for _ in range(n):
        engine.enrich(o, h, l, c, v, columns=cols, out=sub)
    e1.record(st)
    e1.synchronize()
    ms = e0.elapsed_time(e1) / n
    byts = S * T * 8 * (5 + len(cols))
    print(json.dumps({"subset": name, "S": S, "T": T, "ncols": len(cols), "ms": round(ms, 4),
                      "GBps": round(byts / ms / 1e6, 1), "lib": os.environ.get("BQ_LIB_PATH", "default")}), flush=True)
