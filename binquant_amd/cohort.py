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

Nothing reads back to the host, so the whole cohort can be captured once
as a hipGraph (``graphs.CapturedPipeline(process_cohort, ...)``) and
replayed per message; captured, the stages run as four concurrent branches
of the graph (the current stream and three side streams forked from it and
joined before the return; eager calls stay on one stream, see
_COHORT_STREAMS).
Frames share one geometry per call: [S, T5] 5m and [S, T15] 15m panels, the
BTC 15m close index-aligned with the 15m panel (a cohort closes on the same
15-minute grid); the 1h resample's bin count is fixed by T15.
"""

from __future__ import annotations

import torch

from . import engine, signals, strategies

RESAMPLE_AGG = {"open": "first", "high": "max", "low": "min", "close": "last", "volume": "sum"}
HOUR_MS = 3_600_000

# The stages read only the cohort's inputs, so they can run as four
# concurrent branches (the current stream + three side streams forked from it
# and joined back before the return; captured, the joins become graph
# edges). At live shapes most stages are a few hundred waves — a quarter of
# the chip — so overlapping them is what is left to gain on the device:
# 1000 x 400 as a graph 1.03 -> 0.70 ms. Eager calls are bound by the host's
# launches, which the stream switches and record_stream calls lengthen (2.62
# -> 3.66 ms), so by default ("capture") the branches are used only while a
# graph is being captured; True: always, False: never.
_COHORT_STREAMS: bool | str = "capture"
_SIDE: dict[int, list[torch.cuda.Stream]] = {}


def _side_streams(device: torch.device, n: int) -> list[torch.cuda.Stream]:
    idx = device.index if device.index is not None else torch.cuda.current_device()
    if idx not in _SIDE:
        _SIDE[idx] = [torch.cuda.Stream(device=idx) for _ in range(n)]
    return _SIDE[idx][:n]


def process_cohort(o5, h5, l5, c5, v5, o15, h15, l15, c15, v15, ts15, btc_ts15, btc_c15,
                   max_bars: int = 400, exact: bool = True, h1_max_bins: int | None = None) -> dict[str, torch.Tensor]:
    """Device outputs of process_data for a cohort: 5m / 15m panels [S, T5] /
    [S, T15] float64, ts15 [S, T15] int64 open times, btc_ts15 / btc_c15 [T15]
    (index-aligned with the 15m panel). exact=True runs the strategy
    pipelines' bit-exact replays (the live path); False their panel mode.
    h1_max_bins: width of the h1.* arrays (default T15 // 4 + 2, every bin
    of a gap-free 15m grid). pandas emits every empty hour of a gap, so a row
    spanning more hours keeps its NEWEST h1_max_bins bins (bq_resample_tail):
    h1.bins is the count written (<= h1_max_bins, bin h1.bins - 1 is the
    row's latest hour) and h1.dropped the oldest bins left out (0 on a
    gap-free grid). Returns a flat dict of tensors (names prefixed by the
    stage)."""
    S, T15 = c15.shape
    B1 = T15 // 4 + 2 if h1_max_bins is None else int(h1_max_bins)
    btc_c = btc_c15.reshape(-1)

    def frame_5m(out):   # :364-388
        for k, v in engine.enrich(o5, h5, l5, c5, v5).items():
            out[f"e5.{k}"] = v
        for k, v in strategies.activity_burst_features(o5, h5, l5, c5, v5, v5 * c5).items():
            out[f"burst.{k}"] = v

    def frame_15m(out):   # :402-432
        for k, v in engine.enrich(o15, h15, l15, c15, v15).items():
            out[f"e15.{k}"] = v
        bins, res, nbins = engine.resample(ts15, {"open": o15, "high": h15, "low": l15, "close": c15,
                                                  "volume": v15}, RESAMPLE_AGG, HOUR_MS, max_bins=B1, tail=True)
        out["h1.open_time"] = bins
        out["h1.bins"] = nbins.clamp(max=B1)
        out["h1.dropped"] = (nbins - B1).clamp(min=0)
        for k, v in res.items():
            out[f"h1.{k}"] = v
        bc = engine.beta_corr(c15, btc_c15, 50)
        out["btc.beta"], out["btc.corr"] = bc["beta"][:, -1], bc["corr"][:, -1]
        # pct_change(96) with pandas' default pad fill (context_evaluator.py:427-430)
        out["btc.change_24h"] = engine.pct_change(btc_c15.reshape(1, -1), 96)[0, -1:] * 100.0

    def context(out):   # klines_provider.py:181-199
        part, last = engine.context_partials(h15, l15, c15, max_bars=max_bars, last=True)
        out["context.partial"] = part
        for k, v in last.items():
            out[f"context.{k}"] = v

    def pump(out):   # :445-499
        for k, v in strategies.pump_score_features(o15, h15, l15, c15, v15, btc_c, exact=exact).items():
            out[f"pump.{k}"] = v

    def spike(out):
        for k, v in strategies.failed_spike_features(o15, h15, l15, c15, v15, v15 * c15, exact=exact).items():
            out[f"spike.{k}"] = v

    def top(out):
        feats, status = signals.top_gainer_features(o15, h15, l15, c15, v15, v15 * c15)
        for k, v in feats.items():
            out[f"top.{k}"] = v
        out["top.status"] = status

    def lead(out):
        for k, v in signals.gradual_gainer_leadership(ts15, c15, btc_ts15, btc_c).items():
            out[f"lead.{k}"] = v

    order = (frame_5m, frame_15m, context, pump, spike, top, lead)
    parts = {f: {} for f in order}
    branches = _COHORT_STREAMS is True or (_COHORT_STREAMS == "capture"
                                            and torch.cuda.is_current_stream_capturing())
    if not branches:
        for f in order:
            f(parts[f])
    else:
        main = torch.cuda.current_stream(c15.device)
        sides = _side_streams(c15.device, 3)
        groups = ((main, (frame_5m, lead)), (sides[0], (frame_15m, context)), (sides[1], (pump, top)),
                  (sides[2], (spike,)))
        for st in sides:
            st.wait_stream(main)
        for st, fs in groups:
            with torch.cuda.stream(st):
                for f in fs:
                    f(parts[f])
        for st in sides:
            main.wait_stream(st)
        for st, fs in groups[1:]:   # outputs made on a side stream are used on the caller's
            for f in fs:
                for v in parts[f].values():
                    v.record_stream(main)
    out: dict[str, torch.Tensor] = {}
    for f in order:
        out.update(parts[f])
    return out
