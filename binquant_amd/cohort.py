"""One message cohort on the device: ContextEvaluator.process_data
(producers/context_evaluator.py:347-512) for every symbol of a 15-minute
cohort at once.

KlinesProvider.aggregate_data (consumers/klines_provider.py:300-380) hands
process_data one symbol's 5m and 15m frames (plus the BTC 15m frame) per
closed kline, and the accumulator's context refresh runs beside it
(klines_provider.py:181-199). In the reference every symbol of a cohort pays
that path on its own — ~56 ms of pandas per symbol (enrichment
5.1 ms x 2 frames, the store features 2.2, the burst / pump / spike
pipelines 9.1 / 9.8 / 24.3). ``process_cohort`` runs the same device work for
all S symbols of the cohort in one call:

* 5m frame: indicators_enrichment (bq_enrich, the 14 columns, :367-369) and
  ActivityBurstPump's features (:380-388);
* 15m frame: indicators_enrichment (:415), the 1h resample (:403-407, a9),
  dynamic_btc_beta_corr (:424, a11: index-aligned frames) and the BTC
  pct_change(96) (:425-428, a12);
* the context refresh at the cohort's close: the breadth partials of every
  timestamp and the last timestamp's symbol features
  (live_market_context_accumulator.py:95-297, bq_context_partials);
* the 15m strategies' feature pipelines: LiquidationSweepPump,
  FailedSpikeFade, TopGainerEarlyMomentum, GradualGainerRetest's leadership
  (:445-499).

Every launch goes on the current stream and nothing reads back to the host,
so the whole cohort can be captured once as a hipGraph
(``graphs.CapturedPipeline(process_cohort, ...)``) and replayed per message.
Frames share one geometry per call: [S, T5] 5m and [S, T15] 15m panels, the
BTC 15m close index-aligned with the 15m panel (a cohort closes on the same
15-minute grid); the 1h resample's bin count is fixed by T15.
"""

from __future__ import annotations

import torch

from . import engine, signals, strategies

RESAMPLE_AGG = {"open": "first", "high": "max", "low": "min", "close": "last", "volume": "sum"}
HOUR_MS = 3_600_000


def process_cohort(o5, h5, l5, c5, v5, o15, h15, l15, c15, v15, ts15, btc_ts15, btc_c15,
                   max_bars: int = 400, exact: bool = True) -> dict[str, torch.Tensor]:
    """Device outputs of process_data for a cohort: 5m / 15m panels [S, T5] /
    [S, T15] float64, ts15 [S, T15] int64 open times, btc_ts15 / btc_c15 [T15]
    (index-aligned with the 15m panel). exact=True runs the strategy
    pipelines' bit-exact replays (the live path); False their panel mode.
    Returns a flat dict of tensors (names prefixed by the stage)."""
    S, T15 = c15.shape
    out: dict[str, torch.Tensor] = {}
    # ---- 5m frame (:364-388)
    for k, v in engine.enrich(o5, h5, l5, c5, v5).items():
        out[f"e5.{k}"] = v
    for k, v in strategies.activity_burst_features(o5, h5, l5, c5, v5, v5 * c5).items():
        out[f"burst.{k}"] = v
    # ---- 15m frame (:402-432)
    for k, v in engine.enrich(o15, h15, l15, c15, v15).items():
        out[f"e15.{k}"] = v
    bins, res, nbins = engine.resample(ts15, {"open": o15, "high": h15, "low": l15, "close": c15, "volume": v15},
                                       RESAMPLE_AGG, HOUR_MS, max_bins=T15 // 4 + 2)
    out["h1.open_time"] = bins
    out["h1.bins"] = nbins
    for k, v in res.items():
        out[f"h1.{k}"] = v
    bc = engine.beta_corr(c15, btc_c15, 50)
    out["btc.beta"], out["btc.corr"] = bc["beta"][:, -1], bc["corr"][:, -1]
    out["btc.change_24h"] = ((btc_c15[-1] / btc_c15[-97] - 1.0) * 100.0).reshape(1) if T15 > 96 else \
        torch.full((1,), float("nan"), dtype=torch.float64, device=c15.device)
    # ---- context refresh at the cohort's close (klines_provider.py:181-199)
    part, last = engine.context_partials(h15, l15, c15, max_bars=max_bars, last=True)
    out["context.partial"] = part
    for k, v in last.items():
        out[f"context.{k}"] = v
    # ---- 15m strategies (:445-499)
    btc_c = btc_c15.reshape(-1)
    for k, v in strategies.pump_score_features(o15, h15, l15, c15, v15, btc_c, exact=exact).items():
        out[f"pump.{k}"] = v
    for k, v in strategies.failed_spike_features(o15, h15, l15, c15, v15, v15 * c15, exact=exact).items():
        out[f"spike.{k}"] = v
    top, status = signals.top_gainer_features(o15, h15, l15, c15, v15, v15 * c15)
    for k, v in top.items():
        out[f"top.{k}"] = v
    out["top.status"] = status
    for k, v in signals.gradual_gainer_leadership(ts15, c15, btc_ts15, btc_c).items():
        out[f"lead.{k}"] = v
    return out
