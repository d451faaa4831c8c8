"""Batched strategy feature pipelines on the GPU ([S, T] panels).

* activity_burst_features — ActivityBurstPump.compute_indicators
  (strategies/activity_burst_pump.py:51-158), the volume/price-burst detector.
* pump_score_features — LiquidationSweepPump.compute_pump_score
  (strategies/liquidation_sweep_pump.py:195-269).
* failed_spike_features — FailedSpikeFade.detect
  (strategies/failed_spike_fade.py:533-544): base / early features, the
  whole-series auto-calibration, labels, cooldown and streaks.

The order statistics and recurrences run in the hand-written kernels of
bq_rolling.hip (rolling median / quantile / mean / sum / var / std / max / min
with pandas' NaN and min_periods rules; ewm with NaN-gap decay) and
bq_select.hip (whole-series numpy quantile, sequential cooldown); the
element-wise glue is
device tensor arithmetic in the reference's operation order. Every column
keeps the reference's name; booleans are returned as torch.bool.
"""

from __future__ import annotations

from dataclasses import dataclass

import torch

from . import engine

NAN = float("nan")


def _shift(x: torch.Tensor, n: int) -> torch.Tensor:
    """pandas Series.shift(n) along T (negative n shifts backwards)."""
    out = torch.full_like(x, NAN)
    T = x.shape[-1]
    if 0 <= n < T:
        out[..., n:] = x[..., : T - n]
    elif -T < n < 0:
        out[..., : T + n] = x[..., -n:]
    return out


def _diff(x: torch.Tensor, n: int = 1) -> torch.Tensor:
    """Series.diff(n)."""
    return x - _shift(x, n)


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
    """Forward fill along T, sync-free (no data-dependent host branch, so a
    pipeline using it can be captured in a hipGraph)."""
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
    R = engine.Roll
    up = (c > _shift(c, 1)).to(torch.float64)
    specs = [R(v, bw - 1, "median", min_periods=bw - 1, shift=2), R(up, 3, "sum", min_periods=3)]
    if has_q:
        specs.append(R(qv, bw - 1, "median", min_periods=bw - 1, shift=2))
    res = engine.rolling_many(*specs)
    out["baseline_volume"] = res[0]
    out["baseline_volume_safe"] = _clip_lower(out["baseline_volume"], p.min_baseline_volume)
    out["volume_ratio"] = v / out["baseline_volume_safe"]
    if has_q:
        out["baseline_quote_volume"] = res[2]
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
    out["recent_up_closes"] = res[1]
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
    R, E = engine.Roll, engine.Ewm
    atr, vmean, hmax, lmin, e20, e50 = engine.rolling_many(
        E(tr, alpha=1 / 14, min_periods=14), R(v, p.volume_lookback, "mean", shift=1),
        R(h, p.compression_bars, "max", shift=1), R(l, p.compression_bars, "min", shift=1),
        E(c, span=20), E(c, span=50),
    )
    out["candidate_atr"] = atr
    out["momentum_3"] = _pct_change(c, p.momentum_bars)
    out["relative_volume"] = v / vmean
    out["pre_breakout_compression"] = (hmax - lmin) / prev
    out["pump_score"] = (
        out["relative_volume"] * _clip_lower(out["momentum_3"], 0.0) / _replace0(out["pre_breakout_compression"])
    )
    out["score_threshold"], out["volume_threshold"] = engine.rolling_many(
        R(out["pump_score"], p.score_lookback, "quantile", q=p.score_quantile, shift=1),
        R(out["relative_volume"], p.score_lookback, "quantile", q=p.score_quantile, shift=1),
    )
    out["score_cross"] = (out["pump_score"] >= out["score_threshold"]) & (
        _shift(out["pump_score"], 1) < _shift(out["score_threshold"], 1)
    )
    out["prior_high"] = hmax
    out["close_location"] = (c - l) / _replace0(h - l)
    out["ema20"] = e20
    out["ema50"] = e50
    out["trend_score"] = (out["ema20"] - out["ema50"]) / out["ema50"]
    out["momentum_atr"] = out["momentum_3"] / (out["candidate_atr"] / c)
    bench = btc_close.reshape(1, -1)
    out["btc_momentum_3"] = _pct_change(bench, p.momentum_bars).expand_as(c)
    be20, be50 = engine.rolling_many(E(bench.contiguous(), span=20), E(bench.contiguous(), span=50))
    out["btc_trend_score"] = ((be20 - be50) / be50).expand_as(c)
    out["relative_strength"] = out["momentum_3"] - out["btc_momentum_3"]
    return out


@dataclass
class SpikeParams:
    """FailedSpikeFade thresholds (strategies/failed_spike_fade.py:66-91) that
    detect() uses; the auto_calibrate defaults of :229-235."""

    volume_cluster_min_ratio: float = 1.6
    volume_cluster_window: int = 8
    volume_cluster_min_count: int = 2
    volume_cluster_label_mode: str = "last"   # last | all | first
    price_break_base_threshold: float = 0.03
    price_break_dynamic_q: float = 0.85
    price_break_use_dynamic: bool = True
    cumulative_price_window: int = 3
    cumulative_price_threshold: float = 0.025
    accel_volume_deriv_window: int = 3
    accel_volume_deriv_min: float = 0.45
    accel_price_change_min: float = 0.015
    require_both_patterns: bool = False
    post_spike_cooldown_bars: int = 8
    require_bullish_spike: bool = True
    body_size_pct_min: float = 0.005
    base_window: int = 12
    streak_length: int = 3
    # auto_calibrate(volume_quantile, price_base_floor_quantile, min_volume_ratio, min_price_abs_floor)
    volume_quantile: float = 0.97
    price_base_floor_quantile: float = 0.75
    min_volume_ratio: float = 1.15
    min_price_abs_floor: float = 0.015


def failed_spike_features(o, h, l, c, v, qv, p: SpikeParams | None = None) -> dict[str, torch.Tensor]:
    """FailedSpikeFade.detect on an [S, T] panel (one row per symbol's df_15m,
    RangeIndex). Integer columns come back as torch.bool (label_pre /
    label_short_pre likewise); 'volume_cluster_min_ratio' and
    'price_break_base_threshold' hold the per-symbol auto-calibrated values."""
    p = p or SpikeParams()
    eps = 1e-6
    out: dict[str, torch.Tensor] = {}
    w = p.base_window
    # ---- compute_base_features (:260-322) ----
    pc = _pct_change(c, 1)
    pca = pc.abs()
    out["price_change"] = pc
    out["price_change_abs"] = pca
    body = (c - o).abs()
    out["body_size"] = body
    out["body_size_pct"] = body / (o + eps)
    out["upper_wick"] = h - torch.fmax(c, o)          # DataFrame.max(axis=1) skips NaN
    out["lower_wick"] = torch.fmin(c, o) - l
    out["upper_wick_ratio"] = out["upper_wick"] / (body + eps)
    out["lower_wick_ratio"] = out["lower_wick"] / (body + eps)
    out["total_range"] = h - l
    out["range_pct"] = out["total_range"] / (o + eps)
    out["is_bullish"] = c > o
    out["close_open_ratio"] = (c - o) / (o + eps)
    # every rolling series that depends only on the inputs: ONE batched call
    R, E = engine.Roll, engine.Ewm  # noqa: F841
    bsp = out["body_size_pct"]
    cw, n = p.cumulative_price_window, p.streak_length
    neg_pc = torch.where(pc > 0, torch.zeros_like(pc), pc).abs()   # clip(upper=0).abs(), NaN stays
    specs = [R(c, w, "mean"), R(c, w, "std"), R(v, w, "mean"), R(v, w, "std"), R(qv, w, "mean"),
             R(c, 8, "std"), R(c, 20, "std"), R(pc, 2, "sum"), R(pc, 3, "sum"),
             R((pc > 0).to(torch.float64), 5, "sum"), R(pca, 5, "sum"), R(bsp, 10, "mean"), R(bsp, 10, "std"),
             R((c > o).to(torch.float64), n, "sum"), R((c < o).to(torch.float64), n, "sum")]
    if cw > 1:
        specs += [R(_clip_lower(pc, 0.0), cw, "sum"), R(neg_pc, cw, "sum")]
    if p.price_break_use_dynamic:
        specs.append(R(pca, 60, "quantile", q=p.price_break_dynamic_q, min_periods=20))
    res = engine.rolling_many(*specs)
    (price_ma, price_std, volume_ma, volume_std, qv_ma, s8, s20, pc2, pc3, pos5, abs5, bsp_ma, bsp_sd, green,
     red) = res[:15]
    cum_pos, cum_neg = (res[15], res[16]) if cw > 1 else (None, None)
    dyn = res[-1] if p.price_break_use_dynamic else None
    out["price_ma"] = price_ma
    out["price_std"] = price_std
    out["price_zscore"] = (c - out["price_ma"]) / (out["price_std"] + eps)
    out["volume_ma"] = volume_ma
    vr = v / (out["volume_ma"] + eps)
    out["volume_ratio"] = vr
    out["volume_zscore"] = (v - out["volume_ma"]) / (volume_std + eps)
    out["quote_volume_ma"] = qv_ma
    out["quote_volume_ratio"] = qv / (out["quote_volume_ma"] + eps)
    out["momentum_3"] = _pct_change(c, 3)
    out["momentum_5"] = _pct_change(c, 5)
    out["close_to_high"] = (h - c) / (h + eps)
    out["close_to_low"] = (c - l + eps) / (c + eps)
    # ---- auto_calibrate (:229-257): whole-series np.quantile of the dropna'd columns ----
    qv_thr = engine.row_quantile(vr, p.volume_quantile).unsqueeze(1)
    qp_thr = engine.row_quantile(pca, p.price_base_floor_quantile).unsqueeze(1)
    skip = torch.isnan(qv_thr) | torch.isnan(qp_thr)      # vols.empty or pcs.empty
    new_vol = torch.where(qv_thr > p.min_volume_ratio, qv_thr, torch.full_like(qv_thr, p.min_volume_ratio))
    new_floor = torch.where(qp_thr > p.min_price_abs_floor, qp_thr, torch.full_like(qp_thr, p.min_price_abs_floor))
    base0 = p.price_break_base_threshold
    new_base = torch.where(new_floor > base0, new_floor, torch.full_like(new_floor, base0))
    vcmr = torch.where(skip, torch.full_like(new_vol, p.volume_cluster_min_ratio), new_vol)
    pbbt = torch.where(skip, torch.full_like(new_base, base0), new_base)
    out["volume_cluster_min_ratio"] = vcmr.squeeze(1)
    out["price_break_base_threshold"] = pbbt.squeeze(1)
    # ---- compute_early_features (:324-357) ----
    out["rolling_price_std_8"] = s8
    out["rolling_price_std_20"] = s20
    out["std_ratio_8_20"] = s8 / (s20 + eps)
    out["vol_ratio_slope_3"] = _diff(vr, 3)
    out["vol_ratio_accel"] = _diff(out["vol_ratio_slope_3"], 1)
    out["pc_1"] = pc
    out["pc_2c"] = pc2
    out["pc_3c"] = pc3
    out["pc_pos_count_5"] = pos5
    out["pc_abs_sum_5"] = abs5
    out["body_size_pct_ma_10"] = bsp_ma
    out["body_size_pct_std_10"] = bsp_sd
    out["body_size_pct_z"] = (bsp - out["body_size_pct_ma_10"]) / (out["body_size_pct_std_10"] + eps)
    out["vol_compression_flag"] = s8 < s20 * 0.6
    # ---- volume_cluster_flag (:360-370) ----
    cond = vr >= vcmr
    # the two series that need the calibrated ratio: one more batched call
    cnt, vmax = engine.rolling_many(
        R(cond.to(torch.float64), p.volume_cluster_window, "sum", min_periods=1),
        R((vr >= vcmr * 0.8).to(torch.float64), max(cw, 1), "max"),
    )
    base = (cnt >= p.volume_cluster_min_count) & cond
    if p.volume_cluster_label_mode == "last":
        nxt = torch.zeros_like(base)
        nxt[:, :-1] = base[:, 1:]
        vcf = base & ~nxt
    elif p.volume_cluster_label_mode == "first":
        prv = torch.zeros_like(base)
        prv[:, 1:] = base[:, :-1]
        vcf = base & ~prv
    else:
        vcf = base
    out["volume_cluster_flag"] = vcf
    # ---- price_break_flag (:372-400), auto_tune off ----
    if p.price_break_use_dynamic:
        thr = _ffill(torch.where(torch.isnan(dyn), dyn, torch.maximum(pbbt.expand_as(dyn), dyn)))
    else:
        thr = pbbt.expand_as(pca).clone()
    out["price_break_flag"] = pca >= thr
    out["price_break_threshold_series"] = thr
    # ---- cumulative_price_break_flag (:402-421) ----
    cw = p.cumulative_price_window
    if cw <= 1:
        cum_f = torch.zeros_like(cond)
        cum_s = torch.zeros_like(cond)
    else:
        vol_cond = torch.isnan(vmax) | (vmax != 0)          # .astype(bool): NaN -> True
        cum_f = (cum_pos >= p.cumulative_price_threshold) & vol_cond
        cum_s = (cum_neg >= p.cumulative_price_threshold) & vol_cond
    out["cumulative_price_break_flag"] = cum_f
    out["cumulative_price_break_short_flag"] = cum_s
    # ---- acceleration_flag (:423-444) ----
    vd = vr - _shift(vr, p.accel_volume_deriv_window)
    acc = (vd >= p.accel_volume_deriv_min) & (pca >= p.accel_price_change_min)
    out["accel_spike_flag"] = acc & (pc > 0)
    out["accel_spike_short_flag"] = acc & (pc < 0)
    # ---- apply_preliminary_label (:446-488) ----
    if p.require_both_patterns:
        combo = vcf & out["price_break_flag"]
    else:
        combo = vcf | out["price_break_flag"]
    label_pre = combo | cum_f | out["accel_spike_flag"]
    if p.require_bullish_spike:
        label_pre = label_pre & out["is_bullish"]
    if p.body_size_pct_min > 0:
        label_pre = label_pre & (bsp >= p.body_size_pct_min)
    label_short_pre = (combo | cum_s | out["accel_spike_short_flag"]) & (c < o)
    if p.body_size_pct_min > 0:
        label_short_pre = label_short_pre & (bsp >= p.body_size_pct_min)
    out["label_pre"] = label_pre
    out["label_short_pre"] = label_short_pre
    # ---- compute_early_proba (:490-493): disabled in the reference ----
    out["early_spike_proba"] = torch.full_like(c, NAN)
    out["early_proba_aug_flag"] = torch.zeros_like(label_pre)
    # ---- apply_cooldown (:495-520) ----
    if p.post_spike_cooldown_bars <= 0:
        out["label"], out["suppressed_label"] = label_pre.clone(), torch.zeros_like(label_pre)
        out["label_short"], out["suppressed_label_short"] = label_short_pre.clone(), torch.zeros_like(label_pre)
    else:
        out["label"], out["suppressed_label"] = engine.cooldown(label_pre, p.post_spike_cooldown_bars)
        out["label_short"], out["suppressed_label_short"] = engine.cooldown(label_short_pre,
                                                                            p.post_spike_cooldown_bars)
    # ---- detect_streaks (:522-531) ----
    out["upward"] = green >= n
    out["downward"] = red >= n
    return out
