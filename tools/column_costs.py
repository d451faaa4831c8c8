"""Marginal kernel time per output-column group (diagnostic, GPU)."""
import sys, os, json
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from binquant_amd import engine
from binquant_amd._lib import ENRICH_COLUMNS
from binquant_amd.synth import device_panel

S, T = 12500, 10000
p = device_panel(S, T, seed=1)
groups = {
    "all": ENRICH_COLUMNS,
    "ma7": ("ma_7",),
    "mas": ("ma_7", "ma_25", "ma_100"),
    "ema": ("ema20",),
    "emas+macd": ("macd", "macd_signal", "ema20", "ema50"),
    "bb": ("bb_upper", "bb_mid", "bb_lower"),
    "rsi": ("rsi",),
    "atr": ("ATR",),
    "twap": ("twap",),
    "mfi": ("mfi",),
    "all_but_rsi_mfi": tuple(c for c in ENRICH_COLUMNS if c not in ("rsi", "mfi")),
}
out = {k: torch.empty((S, T), dtype=torch.float64, device="cuda") for k in ENRICH_COLUMNS}
res = {}
for name, cols in groups.items():
    o = {c: out[c] for c in cols}
    for _ in range(2):
        engine.enrich(p["open"], p["high"], p["low"], p["close"], p["volume"], columns=cols, out=o)
    torch.cuda.synchronize()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    ev[0].record()
    for _ in range(10):
        engine.enrich(p["open"], p["high"], p["low"], p["close"], p["volume"], columns=cols, out=o)
    ev[1].record()
    torch.cuda.synchronize()
    ms = ev[0].elapsed_time(ev[1]) / 10
    gb = S * T * 8 * (5 + len(cols)) / 1e9
    res[name] = dict(ms=round(ms, 3), cols=len(cols), GBps=round(gb / ms * 1e3, 1))
    print(name, res[name], flush=True)
json.dump(res, open("gpurun_out/column_costs.json", "w"), indent=1)
