"""Batched strategy feature pipelines on the GPU ([S, T] panels).

* activity_burst_features — ActivityBurstPump.compute_indicators
  (strategies/activity_burst_pump.py:51-158), the volume/price-burst detector.
* pump_score_features — LiquidationSweepPump.compute_pump_score
  (strategies/liquidation_sweep_pump.py:195-269).
* failed_spike_features — FailedSpikeFade.detect
  (strategies/failed_spike_fade.py:533-544): base / early features, the
  whole-series auto-calibration, labels, cooldown and streaks.

Each pipeline is a few stages: the order statistics, recurrences and
forward fills run in the kernels of bq_rolling.hip (rolling median / quantile
/ mean / sum / var / std / max / min with pandas' NaN and min_periods rules;
ewm with NaN-gap decay; ffill), batched per stage; the element-wise glue
between them is one fused program per stage (binquant_amd.fused,
bq_fused_eval) written in the reference's operation order, so every column
equals the unfused arithmetic bit for bit. bq_select.hip adds the
whole-series numpy quantile and the sequential cooldown. Every column keeps
the reference's name; booleans are returned as torch.bool.
"""

from __future__ import annotations

import os

from dataclasses import dataclass

import torch

from . import engine
from . import fused as F

NAN = float("nan")
R, E, FF = engine.Roll, engine.Ewm, engine.Ffill


def pct_change_filled(filled: torch.Tensor | F.Ex, periods: int) -> F.Ex:
    """Series.pct_change(periods) with pandas 2.3.3's default fill_method='pad',
    given the forward-filled series (engine.Ffill): ffill(x) / ffill(x).shift(p) - 1
    ([1,2,nan,4,5] -> [nan,1,0,1,0.25])."""
    f = F._as_ex(filled)
    return f / F.shift(f, periods) - 1


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
    if _BURST_FUSED and p.cooldown_bars <= 8:
        return _activity_burst_fused(o, h, l, c, v, qv, p)
    O, H, L, C, V = (F.inp(t) for t in (o, h, l, c, v))
    Q = F.inp(qv) if has_q else None
    mb = p.min_baseline_volume
    # volume.shift(2).rolling(bw - 1, min_periods=bw - 1).median()   (:58-63)
    up = F.run({"up": (C > F.shift(C, 1)).float()})["up"]
    specs = [R(v, bw - 1, "median", min_periods=bw - 1, shift=2), R(up, 3, "isum", min_periods=3)]
    if has_q:
        specs.append(R(qv, bw - 1, "median", min_periods=bw - 1, shift=2))
    res = engine.rolling_many(*specs)
    e: dict[str, object] = {}
    e["baseline_volume"] = res[0]
    bvs = F.clip_lower(res[0], mb)
    e["baseline_volume_safe"] = bvs
    vr = V / bvs
    e["volume_ratio"] = vr
    if has_q:
        e["baseline_quote_volume"] = res[2]
        bqs = F.clip_lower(res[2], mb)
        e["baseline_quote_volume_safe"] = bqs
        qvr = Q / bqs
        e["quote_volume_ratio"] = qvr
    else:
        qvr = F.const(1.0)
        e["quote_volume_ratio"] = qvr
    prev_close = F.clip_lower(F.shift(C, 1), mb)
    candle_range = F.clip_lower(H - L, mb)
    candle_body = (C - O).abs()
    pj = (C - F.shift(C, 1)) / prev_close
    e["price_jump"] = pj
    rf = candle_range / F.clip_lower(C, mb)
    e["range_frac"] = rf
    bf = candle_body / candle_range
    e["body_frac"] = bf
    cth = (H - C) / candle_range
    e["close_to_high"] = cth
    bull = C > O
    e["is_bullish"] = bull
    e["recent_up_closes"] = res[1]
    e["vol_spike"] = V > (p.volume_multiplier * bvs)
    e["quote_vol_spike"] = Q > (p.quote_volume_multiplier * bqs) if has_q else F.const(True)
    e["price_jump_flag"] = pj > p.price_threshold
    e["range_expansion_flag"] = rf > p.min_range_frac
    e["body_quality_flag"] = bull & (bf > p.min_body_frac) & (cth < p.max_close_to_high)
    min_up = p.min_recent_up_closes if has_q else 1
    e["trend_quality_flag"] = F.inp(res[1]) >= min_up
    pjc = F.clip_lower(pj, 0.0)
    e["activity_burst_score"] = vr * qvr * pjc * (1 + bf) if has_q else vr * pjc
    out = F.run(e)
    if not has_q:
        out["baseline_quote_volume"] = out["baseline_volume"]
        out["baseline_quote_volume_safe"] = out["baseline_volume_safe"]
    # score.shift(1).rolling(80, min_periods=20).quantile(0.92)   (:134-139)
    out["score_threshold"] = engine.rolling(
        out["activity_burst_score"], p.score_lookback, "quantile", q=p.score_quantile,
        min_periods=p.lookback_window, shift=1,
    )
    thr = F.fillna(out["score_threshold"], 0.0)
    flags = [F.inp(out[k]) for k in ("vol_spike", "quote_vol_spike", "price_jump_flag", "range_expansion_flag",
                                     "body_quality_flag", "trend_quality_flag")]
    raw = flags[0] & flags[1] & flags[2] & flags[3] & flags[4] & flags[5] & (F.inp(out["activity_burst_score"]) >= thr)
    rawf = F.run({"raw": raw.float()})["raw"]
    # raw.shift(1).rolling(cooldown, min_periods=1).max().fillna(False)   (:147-152)
    recent = engine.rolling(rawf, p.cooldown_bars, "max", min_periods=1, shift=1)
    out["qualified_signal"] = F.run({"q": F.inp(rawf).bool() & ~(F.fillna(recent, 0.0) > 0)})["q"]
    order = ["baseline_volume", "baseline_volume_safe", "volume_ratio", "baseline_quote_volume",
             "baseline_quote_volume_safe", "quote_volume_ratio", "price_jump", "range_frac", "body_frac",
             "close_to_high", "is_bullish", "recent_up_closes", "vol_spike", "quote_vol_spike", "price_jump_flag",
             "range_expansion_flag", "body_quality_flag", "trend_quality_flag", "activity_burst_score",
             "score_threshold", "qualified_signal"]
    return {k: out[k] for k in order}


def _activity_burst_fused(o, h, l, c, v, qv, p: BurstParams) -> dict[str, torch.Tensor]:
    """activity_burst_features through bq_burst_features / bq_burst_qualify:
    the baseline medians and the score's quantile by bq_rolling_batch, every
    other column in two streaming passes — bit for bit the staged pipeline."""
    has_q = qv is not None
    bw = max(p.lookback_window, 2)
    specs = [R(v, bw - 1, "median", min_periods=bw - 1, shift=2)]
    if has_q:
        specs.append(R(qv, bw - 1, "median", min_periods=bw - 1, shift=2))
    med = engine.rolling_many(*specs)
    bq = med[1] if has_q else None
    cols, all_flags = engine.burst_features(o, h, l, c, v, qv, med[0], bq, p)
    thr = engine.rolling(cols["activity_burst_score"], p.score_lookback, "quantile", q=p.score_quantile,
                         min_periods=p.lookback_window, shift=1)
    out = {"baseline_volume": med[0], "baseline_volume_safe": cols["baseline_volume_safe"],
           "volume_ratio": cols["volume_ratio"], "baseline_quote_volume": bq if has_q else med[0],
           "baseline_quote_volume_safe": cols["baseline_quote_volume_safe"],
           "quote_volume_ratio": cols["quote_volume_ratio"]}
    for k in ("price_jump", "range_frac", "body_frac", "close_to_high", "is_bullish", "recent_up_closes", "vol_spike",
              "quote_vol_spike", "price_jump_flag", "range_expansion_flag", "body_quality_flag", "trend_quality_flag",
              "activity_burst_score"):
        out[k] = cols[k]
    out["score_threshold"] = thr
    out["qualified_signal"] = engine.burst_qualify(cols["activity_burst_score"], thr, all_flags, p.cooldown_bars)
    return out


# activity_burst_features through bq_burst_features (False: the staged
# pipeline; tests compare the two)
_BURST_FUSED = True

def _failed_spike_fused(o, h, l, c, v, qv, p: SpikeParams) -> dict[str, torch.Tensor]:
    """failed_spike_features (panel mode) through bq_spike_base(_std) /
    bq_spike_flags: the close ffill, the base / early features and the five
    rolling std columns in one pass (BQ_SPIKE_STD_IN_PASS=0: the stds as the
    bit-exact replays of pandas' online variance, batched with the ffill), the
    |pct change| quantile and the whole-series calibration, the flags and
    labels in a second pass, then both cooldowns in one launch."""
    eps = 1e-6
    w, n = p.base_window, p.streak_length
    O, C = F.inp(o), F.inp(c)
    if _SPIKE_STD_IN_PASS:   # the five std columns formed in the base pass (reference-shifted window sums)
        (cf,) = engine.rolling_many(FF(c))
        b = engine.spike_base_std(o, h, l, c, v, qv, cf, w, n)   # body_size_pct formed in the pass too
        price_std, volume_std, s8, s20, bsp_sd = (b[k] for k in engine.SPIKE_STD)
    else:                    # the five std columns as the bit-exact replays of pandas' online variance
        bsp = F.run({"bsp": (C - O).abs() / (O + eps)})["bsp"]
        cf, price_std, volume_std, s8, s20, bsp_sd = engine.rolling_many(
            FF(c), R(c, w, "std"), R(v, w, "std"), R(c, 8, "std"), R(c, 20, "std"), R(bsp, 10, "std"))
        b = engine.spike_base(o, h, l, c, v, qv, cf, price_std, volume_std, s8, s20, bsp_sd, w, n,
                              body_size_pct=bsp)
    pca = b["price_change_abs"]
    (dyn,) = engine.rolling_many(R(pca, 60, "quantile", q=p.price_break_dynamic_q, min_periods=20), exact=False)
    vr = b["volume_ratio"]
    qv_thr = engine.row_quantile(vr, p.volume_quantile).unsqueeze(1)
    qp_thr = engine.row_quantile(pca, p.price_base_floor_quantile).unsqueeze(1)
    skip = torch.isnan(qv_thr) | torch.isnan(qp_thr)
    new_vol = torch.where(qv_thr > p.min_volume_ratio, qv_thr, torch.full_like(qv_thr, p.min_volume_ratio))
    new_floor = torch.where(qp_thr > p.min_price_abs_floor, qp_thr, torch.full_like(qp_thr, p.min_price_abs_floor))
    base0 = p.price_break_base_threshold
    new_base = torch.where(new_floor > base0, new_floor, torch.full_like(new_floor, base0))
    vcmr = torch.where(skip, torch.full_like(new_vol, p.volume_cluster_min_ratio), new_vol).contiguous()
    pbbt = torch.where(skip, torch.full_like(new_base, base0), new_base).contiguous()
    S, T = c.shape
    labels = torch.empty((2, S, T), dtype=torch.bool, device=c.device)   # label_pre / label_short_pre
    f = engine.spike_flags(o, c, cf, vr, dyn, vcmr, pbbt, p, labels=labels)
    out: dict[str, torch.Tensor] = {}
    for key in ("price_change", "price_change_abs", "body_size", "body_size_pct", "upper_wick", "lower_wick",
                "upper_wick_ratio", "lower_wick_ratio", "total_range", "range_pct", "is_bullish", "close_open_ratio"):
        out[key] = b[key]
    out["price_ma"] = b["price_ma"]
    out["price_std"] = price_std
    out["price_zscore"] = b["price_zscore"]
    out["volume_ma"] = b["volume_ma"]
    out["volume_ratio"] = vr
    out["volume_zscore"] = b["volume_zscore"]
    out["quote_volume_ma"] = b["quote_volume_ma"]
    for key in ("quote_volume_ratio", "momentum_3", "momentum_5", "close_to_high", "close_to_low"):
        out[key] = b[key]
    out["volume_cluster_min_ratio"] = vcmr.squeeze(1)
    out["price_break_base_threshold"] = pbbt.squeeze(1)
    out["rolling_price_std_8"] = s8
    out["rolling_price_std_20"] = s20
    out["std_ratio_8_20"] = b["std_ratio_8_20"]
    out["vol_ratio_slope_3"] = f["vol_ratio_slope_3"]
    out["vol_ratio_accel"] = f["vol_ratio_accel"]
    out["pc_1"] = b["price_change"]
    for key in ("pc_2c", "pc_3c", "pc_pos_count_5", "pc_abs_sum_5", "body_size_pct_ma_10"):
        out[key] = b[key]
    out["body_size_pct_std_10"] = bsp_sd
    out["body_size_pct_z"] = b["body_size_pct_z"]
    out["vol_compression_flag"] = b["vol_compression_flag"]
    for key in ("volume_cluster_flag", "price_break_flag", "price_break_threshold_series",
                "cumulative_price_break_flag", "cumulative_price_break_short_flag", "accel_spike_flag",
                "accel_spike_short_flag", "label_pre", "label_short_pre", "early_spike_proba",
                "early_proba_aug_flag"):
        out[key] = f[key]
    label_pre_t, label_short_t = f["label_pre"], f["label_short_pre"]
    if p.post_spike_cooldown_bars <= 0:
        out["label"], out["suppressed_label"] = label_pre_t.clone(), torch.zeros_like(label_pre_t)
        out["label_short"], out["suppressed_label_short"] = label_short_t.clone(), torch.zeros_like(label_pre_t)
    else:
        kept, sup = engine.cooldown(labels.view(2 * S, T), p.post_spike_cooldown_bars)   # both in one launch
        kept, sup = kept.view(2, S, T), sup.view(2, S, T)
        out["label"], out["suppressed_label"] = kept[0], sup[0]
        out["label_short"], out["suppressed_label_short"] = kept[1], sup[1]
    out["upward"] = b["upward"]
    out["downward"] = b["downward"]
    return out


# failed_spike_features (panel mode) through bq_spike_base / bq_spike_flags
# (False: the staged pipeline; tests compare the two)
_SPIKE_FUSED = True
# the fused spike path forms its five rolling std columns inside the base pass
# (bq_spike_base_std: two-pass window sums, panel mode) instead of replaying
# pandas' online variance (bq_rolling_batch) ahead of it. exact=True and the
# staged pipeline keep the replays; tests compare the two within pandas' drift.
_SPIKE_STD_IN_PASS = os.environ.get("BQ_SPIKE_STD_IN_PASS", "1") != "0"

# panel mode of pump_score_features through bq_pump_features (False: the staged
# panel pipeline; tests compare the two)
_PUMP_FUSED = True
# the pump pass forms its ewm columns itself (bq_pump_features_ewm) instead of
# reading them from bq_pump_ewm's scans. Measured slower at 12.5k x 2k (2.11
# vs 1.90 ms per row: the three scans sit between the tile's barriers of a
# pass that runs 2 workgroups per CU), so off; tested both ways.
_PUMP_EWM_IN_PASS = False


@dataclass
class PumpParams:
    """LiquidationSweepPump constants used by compute_pump_score
    (strategies/liquidation_sweep_pump.py:92-104)."""

    momentum_bars: int = 3
    volume_lookback: int = 20
    compression_bars: int = 6
    score_lookback: int = 48
    score_quantile: float = 0.80


def pump_score_features(o, h, l, c, v, btc_close, p: PumpParams | None = None,
                        exact: bool = False) -> dict[str, torch.Tensor]:
    """btc_close: [T] benchmark closes already left-merged onto the panel's
    open_time grid (NaN where the benchmark has no candle), as
    `result[["open_time"]].merge(btc_by_open_time, how="left")` yields.
    exact=True: the ewm / rolling-mean columns by the bit-exact replay (the
    live path); default: time-parallel within rounding of pandas (panel mode)."""
    p = p or PumpParams()
    bench = btc_close.reshape(1, -1).contiguous()
    if _PUMP_FUSED and not exact and max(p.volume_lookback, p.compression_bars) < 31 and p.momentum_bars < 32:
        return _pump_score_fused(h, l, c, v, bench, p)
    H, L, C, V = (F.inp(t) for t in (h, l, c, v))
    prev = F.shift(C, 1)
    tr = F.run({"tr": F.fmax(F.fmax(H - L, (H - prev).abs()), (L - prev).abs())})["tr"]   # max(axis=1) skips NaN
    # the benchmark's [1, T] series ride in the panel's batch (one launch)
    atr, vmean, hmax, lmin, e20, e50, cf, bf, be20, be50 = engine.rolling_many(
        E(tr, alpha=1 / 14, min_periods=14), R(v, p.volume_lookback, "mean", shift=1),
        R(h, p.compression_bars, "max", shift=1), R(l, p.compression_bars, "min", shift=1),
        E(c, span=20), E(c, span=50), FF(c), FF(bench), E(bench, span=20), E(bench, span=50), exact=exact,
    )
    e: dict[str, object] = {}
    e["candidate_atr"] = atr
    m3 = pct_change_filled(cf, p.momentum_bars)
    e["momentum_3"] = m3
    rv = V / vmean
    e["relative_volume"] = rv
    comp = (F.inp(hmax) - lmin) / prev
    e["pre_breakout_compression"] = comp
    e["pump_score"] = rv * F.clip_lower(m3, 0.0) / F.replace0(comp)
    st = F.run(e)
    thr_s, thr_v = engine.rolling_many(
        R(st["pump_score"], p.score_lookback, "quantile", q=p.score_quantile, shift=1),
        R(st["relative_volume"], p.score_lookback, "quantile", q=p.score_quantile, shift=1),
    )
    PS, TS = F.inp(st["pump_score"]), F.inp(thr_s)
    E20, E50 = F.inp(e20), F.inp(e50)
    bm3 = pct_change_filled(F.inp(bf[0]), p.momentum_bars)   # one series for every symbol
    be50x = F.inp(be50[0])
    e2: dict[str, object] = {
        "score_cross": (PS >= TS) & (F.shift(PS, 1) < F.shift(TS, 1)),
        "close_location": (C - L) / F.replace0(H - L),
        "trend_score": (E20 - E50) / E50,
        "momentum_atr": F.inp(st["momentum_3"]) / (F.inp(atr) / C),
        "btc_momentum_3": bm3,
        "btc_trend_score": (F.inp(be20[0]) - be50x) / be50x,
        "relative_strength": F.inp(st["momentum_3"]) - bm3,
    }
    st2 = F.run(e2, *c.shape)
    out = {
        "candidate_atr": atr, "momentum_3": st["momentum_3"], "relative_volume": st["relative_volume"],
        "pre_breakout_compression": st["pre_breakout_compression"], "pump_score": st["pump_score"],
        "score_threshold": thr_s, "volume_threshold": thr_v, "score_cross": st2["score_cross"], "prior_high": hmax,
        "close_location": st2["close_location"], "ema20": e20, "ema50": e50, "trend_score": st2["trend_score"],
        "momentum_atr": st2["momentum_atr"], "btc_momentum_3": st2["btc_momentum_3"],
        "btc_trend_score": st2["btc_trend_score"], "relative_strength": st2["relative_strength"],
    }
    return out


def _pump_score_fused(h, l, c, v, bench, p: PumpParams) -> dict[str, torch.Tensor]:
    """Panel mode of pump_score_features: the per-symbol ewm columns by
    bq_pump_ewm (the ATR's true range formed in the scan), the benchmark's
    ffill / ewm rows by bq_rolling_batch, every other column but the
    quantiles and score_cross in one pass per row (bq_pump_features: the
    volume mean, the high / low windows and the pad-filled pct_change inside
    the kernel), then the two rolling quantiles and score_cross.
    _PUMP_EWM_IN_PASS: the ewm scans inside the pass (bq_pump_features_ewm)."""
    bf, be20, be50 = engine.rolling_many(FF(bench), E(bench, span=20), E(bench, span=50), exact=False)
    if _PUMP_EWM_IN_PASS:
        st = engine.pump_features_ewm(h, l, c, v, bf[0], be20[0], be50[0], p.momentum_bars, p.volume_lookback,
                                      p.compression_bars)
    else:
        atr, e20, e50, trend = engine.pump_ewm(h, l, c, trend=True)
        st = engine.pump_features(h, l, c, v, atr, e20, e50, bf[0], be20[0], be50[0], p.momentum_bars,
                                  p.volume_lookback, p.compression_bars, trend_score=trend)
    # the two quantiles in one launch, score_cross formed in the score's steps
    (thr_s, thr_v), (cross,) = engine.rolling_many(   # panel mode: packed-key order statistics (within 2^-45)
        R(st["pump_score"], p.score_lookback, "quantile", q=p.score_quantile, shift=1),
        R(st["relative_volume"], p.score_lookback, "quantile", q=p.score_quantile, shift=1), exact=False, cross=(0,),
    )
    out = {k: st[k] for k in ("candidate_atr", "momentum_3", "relative_volume", "pre_breakout_compression",
                              "pump_score")}
    out.update(score_threshold=thr_s, volume_threshold=thr_v, score_cross=cross)
    for k in ("prior_high", "close_location", "ema20", "ema50", "trend_score", "momentum_atr", "btc_momentum_3",
              "btc_trend_score", "relative_strength"):
        out[k] = st[k]
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


def failed_spike_features(o, h, l, c, v, qv, p: SpikeParams | None = None,
                          exact: bool = False) -> dict[str, torch.Tensor]:
    """FailedSpikeFade.detect on an [S, T] panel (one row per symbol's df_15m,
    RangeIndex). Integer columns come back as torch.bool (label_pre /
    label_short_pre likewise); 'volume_cluster_min_ratio' and
    'price_break_base_threshold' hold the per-symbol auto-calibrated values.
    exact=True: the rolling sums / means / stds by the bit-exact replay (the
    live path); default: panel mode, within rounding of pandas — the fused
    passes form the five rolling std columns from window sums about an
    in-window reference (the exact window std to rounding, where pandas'
    online variance may drift; BQ_SPIKE_STD_IN_PASS=0 keeps the replay)."""
    p = p or SpikeParams()
    eps = 1e-6
    S, T = c.shape
    w = p.base_window
    if (_SPIKE_FUSED and not exact and p.price_break_use_dynamic and 2 <= p.cumulative_price_window <= 30
            and max(w, p.streak_length, p.volume_cluster_window, p.accel_volume_deriv_window) <= 30
            and p.volume_cluster_label_mode in ("last", "first", "all")):
        return _failed_spike_fused(o, h, l, c, v, qv, p)
    O, H, L, C, V, Q = (F.inp(t) for t in (o, h, l, c, v, qv))
    # ---- compute_base_features (:260-322) ----
    (cf,) = engine.rolling_many(FF(c))
    pc = pct_change_filled(cf, 1)
    pca = pc.abs()
    body = (C - O).abs()
    bsp = body / (O + eps)
    e: dict[str, object] = {
        "price_change": pc, "price_change_abs": pca, "body_size": body, "body_size_pct": bsp,
        "upper_wick": H - F.fmax(C, O),          # DataFrame.max(axis=1) skips NaN
        "lower_wick": F.fmin(C, O) - L,
    }
    e["upper_wick_ratio"] = e["upper_wick"] / (body + eps)
    e["lower_wick_ratio"] = e["lower_wick"] / (body + eps)
    e["total_range"] = H - L
    e["range_pct"] = e["total_range"] / (O + eps)
    e["is_bullish"] = C > O
    e["close_open_ratio"] = (C - O) / (O + eps)
    cw, n = p.cumulative_price_window, p.streak_length
    # the rolling operands that are element-wise expressions
    e["_pos"] = (pc > 0).float()
    e["_green"] = (C > O).float()
    e["_red"] = (C < O).float()
    if cw > 1:
        e["_clip_pos"] = F.clip_lower(pc, 0.0)
        e["_neg"] = F.where(pc > 0, 0.0, pc).abs()   # clip(upper=0).abs(), NaN stays
    b = F.run(e)
    # every rolling series that depends only on the inputs: ONE batched call
    specs = [R(c, w, "mean"), R(c, w, "std"), R(v, w, "mean"), R(v, w, "std"), R(qv, w, "mean"),
             R(c, 8, "std"), R(c, 20, "std"), R(b["price_change"], 2, "sum"), R(b["price_change"], 3, "sum"),
             R(b["_pos"], 5, "isum"), R(b["price_change_abs"], 5, "sum"), R(b["body_size_pct"], 10, "mean"),
             R(b["body_size_pct"], 10, "std"), R(b["_green"], n, "isum"), R(b["_red"], n, "isum")]
    if cw > 1:
        specs += [R(b["_clip_pos"], cw, "sum"), R(b["_neg"], cw, "sum")]
    if p.price_break_use_dynamic:
        specs.append(R(b["price_change_abs"], 60, "quantile", q=p.price_break_dynamic_q, min_periods=20))
    res = engine.rolling_many(*specs, exact=exact)
    (price_ma, price_std, volume_ma, volume_std, qv_ma, s8, s20, pc2, pc3, pos5, abs5, bsp_ma, bsp_sd, green,
     red) = res[:15]
    cum_pos, cum_neg = (res[15], res[16]) if cw > 1 else (None, None)
    dyn = res[-1] if p.price_break_use_dynamic else None
    VR = V / (F.inp(volume_ma) + eps)
    S8, S20 = F.inp(s8), F.inp(s20)
    BSP = F.inp(b["body_size_pct"])
    e2: dict[str, object] = {
        "price_zscore": (C - price_ma) / (F.inp(price_std) + eps),
        "volume_ratio": VR,
        "volume_zscore": (V - volume_ma) / (F.inp(volume_std) + eps),
        "quote_volume_ratio": Q / (F.inp(qv_ma) + eps),
        "momentum_3": pct_change_filled(cf, 3),
        "momentum_5": pct_change_filled(cf, 5),
        "close_to_high": (H - C) / (H + eps),
        "close_to_low": (C - L + eps) / (C + eps),
        "std_ratio_8_20": S8 / (S20 + eps),
        "body_size_pct_z": (BSP - bsp_ma) / (F.inp(bsp_sd) + eps),
        "vol_compression_flag": S8 < S20 * 0.6,
    }
    m = F.run(e2)
    # ---- auto_calibrate (:229-257): whole-series np.quantile of the dropna'd columns ----
    vr = m["volume_ratio"]
    qv_thr = engine.row_quantile(vr, p.volume_quantile).unsqueeze(1)
    qp_thr = engine.row_quantile(b["price_change_abs"], p.price_base_floor_quantile).unsqueeze(1)
    skip = torch.isnan(qv_thr) | torch.isnan(qp_thr)      # vols.empty or pcs.empty
    new_vol = torch.where(qv_thr > p.min_volume_ratio, qv_thr, torch.full_like(qv_thr, p.min_volume_ratio))
    new_floor = torch.where(qp_thr > p.min_price_abs_floor, qp_thr, torch.full_like(qp_thr, p.min_price_abs_floor))
    base0 = p.price_break_base_threshold
    new_base = torch.where(new_floor > base0, new_floor, torch.full_like(new_floor, base0))
    vcmr = torch.where(skip, torch.full_like(new_vol, p.volume_cluster_min_ratio), new_vol).contiguous()
    pbbt = torch.where(skip, torch.full_like(new_base, base0), new_base).contiguous()
    # ---- compute_early_features (:324-357) and the flag operands ----
    VRm, VC, PB = F.inp(vr), F.inp(vcmr), F.inp(pbbt)
    cond = VRm >= VC
    e3: dict[str, object] = {
        "vol_ratio_slope_3": F.diff(VRm, 3),
        "vol_ratio_accel": F.diff(F.diff(VRm, 3), 1),
        "_cond": cond.float(),
        "_cond8": (VRm >= VC * 0.8).float(),
    }
    if p.price_break_use_dynamic:
        D = F.inp(dyn)
        e3["_thr_pre"] = F.where(F.isnan(D), D, F.maximum(PB, D))
    k = F.run(e3, S, T)
    # ---- volume_cluster_flag (:360-370), the dynamic threshold's ffill (:372-400) ----
    specs2 = [R(k["_cond"], p.volume_cluster_window, "isum", min_periods=1),
              R(k["_cond8"], max(cw, 1), "max")]
    if p.price_break_use_dynamic:
        specs2.append(FF(k["_thr_pre"]))
    res2 = engine.rolling_many(*specs2)
    cnt, vmax = res2[0], res2[1]
    THR = F.inp(res2[2]) if p.price_break_use_dynamic else PB
    base = (F.inp(cnt) >= p.volume_cluster_min_count) & cond
    if p.volume_cluster_label_mode == "last":
        vcf = base & ~F.shift(base, -1)
    elif p.volume_cluster_label_mode == "first":
        vcf = base & ~F.shift(base, 1)
    else:
        vcf = base
    PCA, PC = F.inp(b["price_change_abs"]), F.inp(b["price_change"])
    pbf = PCA >= THR
    # ---- cumulative_price_break_flag (:402-421) ----
    if cw <= 1:
        cum_f = cum_s = F.const(False)
    else:
        VM = F.inp(vmax)
        vol_cond = F.isnan(VM) | (VM != 0)          # .astype(bool): NaN -> True
        cum_f = (F.inp(cum_pos) >= p.cumulative_price_threshold) & vol_cond
        cum_s = (F.inp(cum_neg) >= p.cumulative_price_threshold) & vol_cond
    # ---- acceleration_flag (:423-444) ----
    vd = VRm - F.shift(VRm, p.accel_volume_deriv_window)
    acc = (vd >= p.accel_volume_deriv_min) & (PCA >= p.accel_price_change_min)
    acc_l = acc & (PC > 0)
    acc_s = acc & (PC < 0)
    # ---- apply_preliminary_label (:446-488) ----
    combo = (vcf & pbf) if p.require_both_patterns else (vcf | pbf)
    label_pre = combo | cum_f | acc_l
    if p.require_bullish_spike:
        label_pre = label_pre & F.inp(b["is_bullish"])
    if p.body_size_pct_min > 0:
        label_pre = label_pre & (BSP >= p.body_size_pct_min)
    label_short_pre = (combo | cum_s | acc_s) & (C < O)
    if p.body_size_pct_min > 0:
        label_short_pre = label_short_pre & (BSP >= p.body_size_pct_min)
    e4: dict[str, object] = {
        "volume_cluster_flag": vcf, "price_break_flag": pbf,
        "price_break_threshold_series": THR,
        "cumulative_price_break_flag": cum_f, "cumulative_price_break_short_flag": cum_s,
        "accel_spike_flag": acc_l, "accel_spike_short_flag": acc_s,
        "label_pre": label_pre, "label_short_pre": label_short_pre,
        "upward": F.inp(green) >= n, "downward": F.inp(red) >= n,
        "early_spike_proba": F.const(NAN), "early_proba_aug_flag": F.const(False),
    }
    f = F.run(e4, S, T)
    out: dict[str, torch.Tensor] = {}
    for key in ("price_change", "price_change_abs", "body_size", "body_size_pct", "upper_wick", "lower_wick",
                "upper_wick_ratio", "lower_wick_ratio", "total_range", "range_pct", "is_bullish", "close_open_ratio"):
        out[key] = b[key]
    out["price_ma"] = price_ma
    out["price_std"] = price_std
    out["price_zscore"] = m["price_zscore"]
    out["volume_ma"] = volume_ma
    out["volume_ratio"] = m["volume_ratio"]
    out["volume_zscore"] = m["volume_zscore"]
    out["quote_volume_ma"] = qv_ma
    for key in ("quote_volume_ratio", "momentum_3", "momentum_5", "close_to_high", "close_to_low"):
        out[key] = m[key]
    out["volume_cluster_min_ratio"] = vcmr.squeeze(1)
    out["price_break_base_threshold"] = pbbt.squeeze(1)
    out["rolling_price_std_8"] = s8
    out["rolling_price_std_20"] = s20
    out["std_ratio_8_20"] = m["std_ratio_8_20"]
    out["vol_ratio_slope_3"] = k["vol_ratio_slope_3"]
    out["vol_ratio_accel"] = k["vol_ratio_accel"]
    out["pc_1"] = b["price_change"]
    out["pc_2c"] = pc2
    out["pc_3c"] = pc3
    out["pc_pos_count_5"] = pos5
    out["pc_abs_sum_5"] = abs5
    out["body_size_pct_ma_10"] = bsp_ma
    out["body_size_pct_std_10"] = bsp_sd
    out["body_size_pct_z"] = m["body_size_pct_z"]
    out["vol_compression_flag"] = m["vol_compression_flag"]
    for key in ("volume_cluster_flag", "price_break_flag", "price_break_threshold_series",
                "cumulative_price_break_flag", "cumulative_price_break_short_flag", "accel_spike_flag",
                "accel_spike_short_flag", "label_pre", "label_short_pre", "early_spike_proba",
                "early_proba_aug_flag"):
        out[key] = f[key]
    # ---- apply_cooldown (:495-520) ----
    label_pre_t, label_short_t = f["label_pre"], f["label_short_pre"]
    if p.post_spike_cooldown_bars <= 0:
        out["label"], out["suppressed_label"] = label_pre_t.clone(), torch.zeros_like(label_pre_t)
        out["label_short"], out["suppressed_label_short"] = label_short_t.clone(), torch.zeros_like(label_pre_t)
    else:
        out["label"], out["suppressed_label"] = engine.cooldown(label_pre_t, p.post_spike_cooldown_bars)
        out["label_short"], out["suppressed_label_short"] = engine.cooldown(label_short_t,
                                                                            p.post_spike_cooldown_bars)
    # ---- detect_streaks (:522-531) ----
    out["upward"] = f["upward"]
    out["downward"] = f["downward"]
    return out
