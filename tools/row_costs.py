"""Per-§8-row device timings (diagnostic, GPU): each strategy pipeline and
generic kernel at S symbols x T candles, HIP-event timed on the launch stream.
Usage: python tools/row_costs.py [S] [T]"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch

from binquant_amd import engine, signals, strategies
from binquant_amd.synth import device_panel

S = int(sys.argv[1]) if len(sys.argv) > 1 else 12_500
T = int(sys.argv[2]) if len(sys.argv) > 2 else 2_000
p = device_panel(S, T, seed=3)
o, h, l, c, v = (p[k] for k in ("open", "high", "low", "close", "volume"))
qv = v * c
btc = c[0].clone()
ts = (1_700_000_000_000 + 900_000 * torch.arange(T, device="cuda", dtype=torch.int64)).expand(S, T).contiguous()
atr = engine.enrich(o, h, l, c, v, columns=("ATR",))["ATR"]


def timeit(fn, reps=3):
    fn()
    torch.cuda.synchronize()
    s = torch.cuda.current_stream()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record(s)
    for _ in range(reps):
        fn()
    b.record(s)
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps


rows = {
    "enrich14": lambda: engine.enrich(o, h, l, c, v),
    "market_features": lambda: engine.market_features(h, l, c, max_bars=400),
    "beta_corr": lambda: engine.beta_corr(c, btc, 50),
    "supertrend": lambda: engine.supertrend(h, l, c, atr=atr),
    "rolling_mean20": lambda: engine.rolling(v, 20, "mean"),
    "rolling_median19": lambda: engine.rolling(v, 19, "median", shift=2),
    "rolling_q80": lambda: engine.rolling(v, 80, "quantile", q=0.92, min_periods=20),
    "rolling_std12": lambda: engine.rolling(c, 12, "std"),
    "ewm_alpha": lambda: engine.ewm(c, alpha=1 / 14, min_periods=14),
    "row_quantile": lambda: engine.row_quantile(v, 0.85),
    "activity_burst": lambda: strategies.activity_burst_features(o, h, l, c, v, qv),
    "pump_score": lambda: strategies.pump_score_features(o, h, l, c, v, btc),
    "failed_spike": lambda: strategies.failed_spike_features(o, h, l, c, v, qv),
    "wilder_rsi": lambda: signals.wilder_rsi(c),
    "adx": lambda: signals.adx(h, l, c),
    "zscore": lambda: signals.zscore(c),
    "top_gainer": lambda: signals.top_gainer_features(o, h, l, c, v, qv),
    "resample_1h": lambda: engine.resample(ts, {"open": o, "high": h, "low": l, "close": c, "volume": v},
                                           {"open": "first", "high": "max", "low": "min", "close": "last",
                                            "volume": "sum"}, 3_600_000),
    "align": lambda: engine.align(ts, ts[0], btc),
    "join_returns": lambda: engine.join_returns(ts, c, ts[0], btc, capacity=T),
}
res = {}
for name, fn in rows.items():
    try:
        ms = timeit(fn)
        res[name] = {"ms": round(ms, 4), "Gcandles_s": round(S * T / ms / 1e6, 2)}
    except Exception as e:   # noqa: BLE001
        res[name] = {"error": repr(e)[:200]}
    print(name, res[name], flush=True)
os.makedirs("gpurun_out", exist_ok=True)
json.dump({"S": S, "T": T, "rows": res}, open("gpurun_out/row_costs.json", "w"), indent=1)
