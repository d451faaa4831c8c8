"""Run one §8 row's device path a few times on a synthetic HBM panel — the
program that tools/row_profile.sh traces and counts with rocprofv3.

    python tools/row_prof.py <row> [S T]

Rows (bench.py `rows` names + the headline / C5 legs): enrich, context,
a9_resample_1h, a11_beta_corr, a13_market_features, a17_activity_burst,
a18_pump_score, a19_failed_spike, a20_wilder_rsi, a20_adx, a20_zscore,
a20_leadership, supertrend, f4_btc_join_returns. Default shape 12 500 x 2 000
(the bench's `rows` shape); enrich / context default to 12 500 x 10 000.
Prints the mean HIP-event time per call."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from binquant_amd import engine, signals, strategies  # noqa: E402
from binquant_amd.synth import device_panel  # noqa: E402

name = sys.argv[1]
big = name in ("enrich", "enrich_flat", "context")
S, T = (int(sys.argv[2]), int(sys.argv[3])) if len(sys.argv) > 3 else ((12_500, 10_000) if big else (12_500, 2_000))
p = device_panel(S, T, seed=99)
o, h, l, c, v = (p[k] for k in ("open", "high", "low", "close", "volume"))
qv = v * c
btc = c[0].clone()
ts = (1_700_000_000_000 + 900_000 * torch.arange(T, device=c.device, dtype=torch.int64)).expand(S, T).contiguous()
agg = {"open": "first", "high": "max", "low": "min", "close": "last", "volume": "sum"}
_flat = {}


def flat_out():
    if not _flat:
        _flat.update({k: torch.empty((S, T), dtype=torch.float64, device=c.device) for k in engine.ENRICH_COLUMNS})
    return _flat


calls = {
    "enrich": lambda: engine.enrich(o, h, l, c, v),   # the default outputs: padded pitch on large panels
    "enrich_flat": lambda: engine.enrich(o, h, l, c, v, out=flat_out()),   # contiguous [S, T] outputs
    "context": lambda: engine.context_partials(h, l, c, max_bars=400),
    "a9_resample_1h": lambda: engine.resample(ts, {"open": o, "high": h, "low": l, "close": c, "volume": v}, agg,
                                              3_600_000),
    "a11_beta_corr": lambda: engine.beta_corr(c, btc, 50),
    "a13_market_features": lambda: engine.market_features(h, l, c, max_bars=400),
    "a17_activity_burst": lambda: strategies.activity_burst_features(o, h, l, c, v, qv),
    "a18_pump_score": lambda: strategies.pump_score_features(o, h, l, c, v, btc),
    "a19_failed_spike": lambda: strategies.failed_spike_features(o, h, l, c, v, qv),
    "a20_wilder_rsi": lambda: signals.wilder_rsi(c),
    "a20_adx": lambda: signals.adx(h, l, c),
    "a20_zscore": lambda: signals.zscore(c),
    "a20_leadership": lambda: signals.gradual_gainer_leadership(ts, c, ts[0], btc),
    "supertrend": lambda: engine.supertrend(h, l, c, exact=False),
    "f4_btc_join_returns": lambda: engine.join_returns(ts, c, ts[0], btc, capacity=T),
}
# input bytes read per candle; the algorithmic bytes add every returned output
# at its dtype (bench.py output_bytes)
IN = {"enrich": 40, "enrich_flat": 40, "context": 24, "a9_resample_1h": 48, "a11_beta_corr": 8, "a13_market_features": 24,
      "a17_activity_burst": 48, "a18_pump_score": 32, "a19_failed_spike": 48, "a20_wilder_rsi": 8, "a20_adx": 24,
      "a20_zscore": 8, "a20_leadership": 16, "supertrend": 24, "f4_btc_join_returns": 16}


def output_bytes(res) -> int:
    if isinstance(res, torch.Tensor):
        return res.numel() * res.element_size()
    if isinstance(res, dict):
        return sum(output_bytes(v) for v in res.values())
    if isinstance(res, (tuple, list)):
        return sum(output_bytes(v) for v in res)
    return 0


fn = calls[name]
torch.cuda.synchronize()
time.sleep(0.3)   # a gap in the kernel trace: tools/row_summary.py keeps the kernels after it
bpc = IN[name] + output_bytes(fn()) / (S * T)
fn()
torch.cuda.synchronize()
a, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
reps = 5   # 7 calls in all: PMC sums are divided by CALLS = 7
a.record()
for _ in range(reps):
    fn()
e.record()
torch.cuda.synchronize()
print(f"{name} {S}x{T} ms/call {a.elapsed_time(e) / reps:.4f} alg_bpc {bpc:.3f}", flush=True)
