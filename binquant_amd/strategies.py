"""Batched strategy feature pipelines on the GPU ([S, T] panels).

* activity_burst_features — ActivityBurstPump.compute_indicators
  (strategies/activity_burst_pump.py:51-158), the volume/price-burst detector.
* pump_score_features — LiquidationSweepPump.compute_pump_score
  (strategies/liquidation_sweep_pump.py:195-269).

The order statistics and recurrences run in the hand-written kernels of
bq_rolling.hip (rolling median / quantile / mean / sum / max / min with pandas'
NaN and min_periods rules; ewm with NaN-gap decay); the element-wise glue is
device tensor arithmetic in the reference's operation order. Every column
keeps the reference's name; booleans are returned as torch.bool.
"""

from __future__ import annotations

from dataclasses import dataclass

import torch

from . import engine

NAN = float("nan")


def _shift(x: torch.Tensor, n: int) -> torch.Tensor:
    """pandas Series.shift(n) along T (n >= 0)."""
    out = torch.full_like(x, NAN)
    if n < x.shape[-1]:
        out[..., n:] = x[..., : x.shape[-1] - n]
    return out


def _clip_lower(x: torch.Tensor, lo: float) -> torch.Tensor:
    """Series.clip(lower=lo): NaN stays NaN."""
    return torch.where(x < lo, torch.full_like(x, lo), x)


def _gt(a, b):
    """Elementwise a > b with NaN -> False (pandas comparison semantics)."""
    return a > b


def _replace0(x: torch.Tensor) -> torch.Tensor:
    """Series.replace(0, nan)."""
    return torch.where(x == 0, torch.full_like(x, NAN), x)


def _pct_change(x: torch.Tensor, periods: int) -> torch.Tensor:
    """Series.pct_change(periods) with pandas 2.3.3's default fill_method='pad':
    forward-fill NaNs first ([1,2,nan,4,5] -> [nan,1,0,1,0.25])."""
    f = _ffill(x)
    return f / _shift(f, periods) - 1


def _ffill(x: torch.Tensor) -> torch.Tensor:
    if not torch.isnan(x).any():
        return x
    T = x.shape[-1]
    idx = torch.arange(T, device=x.device).expand_as(x)
    valid = ~torch.isnan(x)
    last = torch.where(valid, idx, torch.zeros_like(idx))
    last = torch.cummax(last, dim=-1).values
    out = torch.gather(x, -1, last)
    # positions before the first observation stay NaN
    seen = torch.cummax(valid.to(torch.int8), dim=-1).values.bool()
    return torch.where(seen, out, torch.full_like(x, NAN))


@dataclass
class BurstParams:
    """ActivityBurstPump constants (strategies/activity_burst_pump.py:38-49)."""

    volume_multiplier: float = 2.75
    quote_volume_multiplier: float = 2.5
    price_threshold: float = 0.01
    lookback_window: int = 20
    min_baseline_volume: float = 1e-8
    min_range_frac: float = 0.012
    min_body_frac: float = 0.45
    max_close_to_high: float = 0.35
    min_recent_up_closes: int = 2
    score_quantile: float = 0.92
    score_lookback: int = 80
    cooldown_bars: int = 3


def activity_burst_features(o, h, l, c, v, qv=None, p: BurstParams | None = None) -> dict[str, torch.Tensor]:
    p = p or BurstParams()
    has_q = qv is not None
    bw = max(p.lookback_window, 2)
    out: dict[str, torch.Tensor] = {}
    # volume.shift(2).rolling(bw - 1, min_periods=bw - 1).median()   (:58-63)
    out["baseline_volume"] = engine.rolling(v, bw - 1, "median", min_periods=bw - 1, shift=2)
    out["baseline_volume_safe"] = _clip_lower(out["baseline_volume"], p.min_baseline_volume)
    out["volume_ratio"] = v / out["baseline_volume_safe"]
    if has_q:
        out["baseline_quote_volume"] = engine.rolling(qv, bw - 1, "median", min_periods=bw - 1, shift=2)
        out["baseline_quote_volume_safe"] = _clip_lower(out["baseline_quote_volume"], p.min_baseline_volume)
        out["quote_volume_ratio"] = qv / out["baseline_quote_volume_safe"]
    else:
        out["baseline_quote_volume"] = out["baseline_volume"]
        out["baseline_quote_volume_safe"] = out["baseline_volume_safe"]
        out["quote_volume_ratio"] = torch.ones_like(c)
    prev_close = _clip_lower(_shift(c, 1), p.min_baseline_volume)
    candle_range = _clip_lower(h - l, p.min_baseline_volume)
    candle_body = (c - o).abs()
    out["price_jump"] = (c - _shift(c, 1)) / prev_close
    out["range_frac"] = candle_range / _clip_lower(c, p.min_baseline_volume)
    out["body_frac"] = candle_body / candle_range
    out["close_to_high"] = (h - c) / candle_range
    out["is_bullish"] = c > o
    up = (c > _shift(c, 1)).to(torch.float64)
    out["recent_up_closes"] = engine.rolling(up, 3, "sum", min_periods=3)
    out["vol_spike"] = v > (p.volume_multiplier * out["baseline_volume_safe"])
    if has_q:
        out["quote_vol_spike"] = qv > (p.quote_volume_multiplier * out["baseline_quote_volume_safe"])
    else:
        out["quote_vol_spike"] = torch.ones_like(c, dtype=torch.bool)
    out["price_jump_flag"] = out["price_jump"] > p.price_threshold
    out["range_expansion_flag"] = out["range_frac"] > p.min_range_frac
    out["body_quality_flag"] = (
        out["is_bullish"] & (out["body_frac"] > p.min_body_frac) & (out["close_to_high"] < p.max_close_to_high)
    )
    min_up = p.min_recent_up_closes if has_q else 1
    out["trend_quality_flag"] = out["recent_up_closes"] >= min_up
    pj = _clip_lower(out["price_jump"], 0.0)
    if has_q:
        out["activity_burst_score"] = out["volume_ratio"] * out["quote_volume_ratio"] * pj * (1 + out["body_frac"])
    else:
        out["activity_burst_score"] = out["volume_ratio"] * pj
    # score.shift(1).rolling(80, min_periods=20).quantile(0.92)   (:134-139)
    out["score_threshold"] = engine.rolling(
        out["activity_burst_score"], p.score_lookback, "quantile", q=p.score_quantile,
        min_periods=p.lookback_window, shift=1,
    )
    thr = torch.nan_to_num(out["score_threshold"], nan=0.0)
    raw = (
        out["vol_spike"] & out["quote_vol_spike"] & out["price_jump_flag"] & out["range_expansion_flag"]
        & out["body_quality_flag"] & out["trend_quality_flag"] & (out["activity_burst_score"] >= thr)
    )
    # raw.shift(1).rolling(cooldown, min_periods=1).max().fillna(False)   (:147-152)
    recent = engine.rolling(raw.to(torch.float64), p.cooldown_bars, "max", min_periods=1, shift=1)
    recent = torch.nan_to_num(recent, nan=0.0) > 0
    out["qualified_signal"] = raw & ~recent
    return out


@dataclass
class PumpParams:
    """LiquidationSweepPump constants used by compute_pump_score
    (strategies/liquidation_sweep_pump.py:92-104)."""

    momentum_bars: int = 3
    volume_lookback: int = 20
    compression_bars: int = 6
    score_lookback: int = 48
    score_quantile: float = 0.80


def pump_score_features(o, h, l, c, v, btc_close, p: PumpParams | None = None) -> dict[str, torch.Tensor]:
    """btc_close: [T] benchmark closes already left-merged onto the panel's
    open_time grid (NaN where the benchmark has no candle), as
    `result[["open_time"]].merge(btc_by_open_time, how="left")` yields."""
    p = p or PumpParams()
    out: dict[str, torch.Tensor] = {}
    prev = _shift(c, 1)
    tr = torch.fmax(torch.fmax(h - l, (h - prev).abs()), (l - prev).abs())   # concat(...).max(axis=1) skips NaN
    out["candidate_atr"] = engine.ewm(tr, alpha=1 / 14, min_periods=14)
    out["momentum_3"] = _pct_change(c, p.momentum_bars)
    out["relative_volume"] = v / engine.rolling(v, p.volume_lookback, "mean", shift=1)
    out["pre_breakout_compression"] = (
        engine.rolling(h, p.compression_bars, "max", shift=1) - engine.rolling(l, p.compression_bars, "min", shift=1)
    ) / prev
    out["pump_score"] = (
        out["relative_volume"] * _clip_lower(out["momentum_3"], 0.0) / _replace0(out["pre_breakout_compression"])
    )
    out["score_threshold"] = engine.rolling(out["pump_score"], p.score_lookback, "quantile", q=p.score_quantile,
                                            shift=1)
    out["score_cross"] = (out["pump_score"] >= out["score_threshold"]) & (
        _shift(out["pump_score"], 1) < _shift(out["score_threshold"], 1)
    )
    out["volume_threshold"] = engine.rolling(out["relative_volume"], p.score_lookback, "quantile",
                                             q=p.score_quantile, shift=1)
    out["prior_high"] = engine.rolling(h, p.compression_bars, "max", shift=1)
    out["close_location"] = (c - l) / _replace0(h - l)
    out["ema20"] = engine.ewm(c, span=20)
    out["ema50"] = engine.ewm(c, span=50)
    out["trend_score"] = (out["ema20"] - out["ema50"]) / out["ema50"]
    out["momentum_atr"] = out["momentum_3"] / (out["candidate_atr"] / c)
    bench = btc_close.reshape(1, -1)
    out["btc_momentum_3"] = _pct_change(bench, p.momentum_bars).expand_as(c)
    be20 = engine.ewm(bench.contiguous(), span=20)
    be50 = engine.ewm(bench.contiguous(), span=50)
    out["btc_trend_score"] = ((be20 - be50) / be50).expand_as(c)
    out["relative_strength"] = out["momentum_3"] - out["btc_momentum_3"]
    return out
