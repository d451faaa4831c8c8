"""Restatement of binquant's live market-context path — TEST INFRASTRUCTURE ONLY.

Follows market_regime/live_market_context_accumulator.py (features :244-297,
context :95-242), market_regime/regime_transitions.py (annotation :25-232) and
shared/utils.py:12-23 (clamp / non_negative / safe_pct). Pinned against golden
vectors produced by the reference modules themselves
(tests/golden/make_golden.py). See oracle/__init__.py.
"""

from __future__ import annotations

from math import ceil

import numpy as np
import pandas as pd

REQUIRED_FRESH_SYMBOLS = 40   # live_market_context_accumulator.py:13
MIN_COVERAGE_RATIO = 0.70     # :14


def clamp(value: float, low: float = -1.0, high: float = 1.0) -> float:   # shared/utils.py:12-13
    return max(low, min(high, float(value)))


def non_negative(value: float) -> float:   # shared/utils.py:16-17
    return max(0.0, float(value))


def safe_pct(current: float, previous: float) -> float:   # shared/utils.py:20-23
    if previous == 0:
        return 0.0
    return (float(current) - float(previous)) / abs(float(previous))


def symbol_features(high, low, close) -> dict | None:
    """_compute_symbol_features (live_market_context_accumulator.py:244-297) on
    one (already timestamp-sorted) history window."""
    closes = pd.Series(np.asarray(close, dtype=np.float64))
    highs = pd.Series(np.asarray(high, dtype=np.float64))
    lows = pd.Series(np.asarray(low, dtype=np.float64))
    if len(closes) < 2:
        return None
    previous_close = closes.shift(1)
    true_range = pd.concat(
        [highs - lows, (highs - previous_close).abs(), (lows - previous_close).abs()], axis=1
    ).max(axis=1)
    ema20 = closes.ewm(span=20, adjust=False, min_periods=1).mean().iloc[-1]
    ema50 = closes.ewm(span=50, adjust=False, min_periods=1).mean().iloc[-1]
    atr = true_range.rolling(14, min_periods=1).mean().iloc[-1]
    mid = closes.rolling(20, min_periods=1).mean()
    std = closes.rolling(20, min_periods=1).std(ddof=0).fillna(0.0)
    bb_upper = mid + (2 * std)
    bb_lower = mid - (2 * std)
    latest_close = float(closes.iloc[-1])
    prev_close = float(closes.iloc[-2])
    atr_pct = float(atr / latest_close) if latest_close else 0.0
    bb_width = float((bb_upper.iloc[-1] - bb_lower.iloc[-1]) / abs(mid.iloc[-1])) if mid.iloc[-1] else 0.0
    trend_score = float((ema20 - ema50) / abs(ema50)) if float(ema50) != 0 else 0.0
    return dict(
        close=latest_close,
        return_pct=safe_pct(latest_close, prev_close),
        ema20=float(ema20),
        ema50=float(ema50),
        above_ema20=latest_close > float(ema20),
        above_ema50=latest_close > float(ema50),
        trend_score=trend_score,
        relative_strength_vs_btc=0.0,
        atr_pct=atr_pct,
        bb_width=bb_width,
    )


def panel_features_at(h, l, c, t: int, max_bars: int) -> dict | None:
    """Features a MarketStateStore(max_bars) history would give at candle t."""
    s = max(0, t - max_bars + 1)
    return symbol_features(h[s : t + 1], l[s : t + 1], c[s : t + 1])


def window_features(h, l, c) -> dict[str, np.ndarray] | None:
    """symbol_features for every row of [S, W] history windows at once (the
    last column is the evaluated candle). The pandas rolling / ewm kernels run
    column by column over a [W, S] frame — the same Cython recursions as the
    per-symbol Series calls of symbol_features — and the scalar tail
    (:273-297) is restated element-wise with the same IEEE operations, so each
    row equals symbol_features(h[s], l[s], c[s]) bit for bit
    (tests/test_oracle_golden.py pins this). For the C5-size checks, where a
    per-symbol pandas loop over 12 500 symbols would take minutes."""
    h, l, c = (np.asarray(x, dtype=np.float64) for x in (h, l, c))
    if c.shape[1] < 2:
        return None
    closes, highs, lows = pd.DataFrame(c.T), pd.DataFrame(h.T), pd.DataFrame(l.T)
    prev = closes.shift(1)
    tr = np.fmax(np.fmax((highs - lows).to_numpy(), (highs - prev).abs().to_numpy()),
                 (lows - prev).abs().to_numpy())   # concat(...).max(axis=1): skip-NaN max
    ema20 = closes.ewm(span=20, adjust=False, min_periods=1).mean().to_numpy()[-1]
    ema50 = closes.ewm(span=50, adjust=False, min_periods=1).mean().to_numpy()[-1]
    atr = pd.DataFrame(tr).rolling(14, min_periods=1).mean().to_numpy()[-1]
    mid = closes.rolling(20, min_periods=1).mean().to_numpy()[-1]
    std = closes.rolling(20, min_periods=1).std(ddof=0).fillna(0.0).to_numpy()[-1]
    upper, lower = mid + (2 * std), mid - (2 * std)
    latest, prev_c = c[:, -1], c[:, -2]
    with np.errstate(divide="ignore", invalid="ignore"):
        atr_pct = np.where(latest != 0, atr / latest, 0.0)
        bb_width = np.where(mid != 0, (upper - lower) / np.abs(mid), 0.0)
        trend = np.where(ema50 != 0, (ema20 - ema50) / np.abs(ema50), 0.0)
        ret = np.where(prev_c == 0, 0.0, (latest - prev_c) / np.abs(prev_c))
    return dict(close=latest, return_pct=ret, ema20=ema20, ema50=ema50, above_ema20=latest > ema20,
                above_ema50=latest > ema50, trend_score=trend, atr_pct=atr_pct, bb_width=bb_width)


def exact_bb_width(closes) -> float:
    """bb_width of _compute_symbol_features (:269-281) over the last
    min(20, n) closes in exact rational arithmetic, rounded once at the end
    (sqrt in float64 of the exactly computed population variance). pandas'
    online roll_var (add / remove Welford steps over the whole history)
    drifts from this by up to ~1e-6 relative when std << mean (a window
    right after a halted stretch); the parity tests use this value to show
    such a deviation is pandas' rounding, not the kernel's."""
    from fractions import Fraction
    from math import sqrt

    w = [Fraction(float(x)) for x in np.asarray(closes, dtype=np.float64)[-20:]]
    m = sum(w) / len(w)
    var = sum((x - m) ** 2 for x in w) / len(w)
    mid = float(m)
    if mid == 0:
        return 0.0
    sd = sqrt(float(var))
    return ((mid + 2 * sd) - (mid - 2 * sd)) / abs(mid)


def panel_window_features_at(h, l, c, t: int, max_bars: int) -> dict[str, np.ndarray] | None:
    """window_features of every symbol of a [S, T] panel at candle t under the
    MarketStateStore(max_bars) cap."""
    s = max(0, t - max_bars + 1)
    return window_features(h[:, s : t + 1], l[:, s : t + 1], c[:, s : t + 1])


def partials_from_features(f: dict[str, np.ndarray]) -> np.ndarray:
    """The _build_context reductions (:135-163) of one timestamp as the
    [10] partial row (count, advancers, decliners, above20, above50, sums of
    return / trend / atr_pct / bb_width, 0), summed in symbol order."""
    ret = f["return_pct"]
    return np.array([ret.size, (ret > 0).sum(), (ret < 0).sum(), f["above_ema20"].sum(), f["above_ema50"].sum(),
                     ret.sum(), f["trend_score"].sum(), f["atr_pct"].sum(), f["bb_width"].sum(), 0.0],
                    dtype=np.float64)


def build_context_from_features(
    feats: dict[str, dict],
    btc_symbol: str,
    total_tracked: int,
    btc_features: dict | None,
    fresh_count: int | None = None,
) -> dict | None:
    """Scalar part of _build_context (:96-242) given per-symbol features."""
    fresh_count = len(feats) if fresh_count is None else fresh_count
    required = max(REQUIRED_FRESH_SYMBOLS, ceil(total_tracked * MIN_COVERAGE_RATIO))
    if fresh_count < required:
        return None
    feats = {k: dict(v) for k, v in feats.items()}
    if btc_symbol in feats:
        btc_features = feats[btc_symbol]
    if btc_features is not None:
        for sym, f in feats.items():
            if sym == btc_symbol:
                continue
            f["relative_strength_vs_btc"] = f["return_pct"] - btc_features["return_pct"]
    n = len(feats)
    if total_tracked == 0 or n < required:
        return None
    vals = list(feats.values())
    return _score(
        n=n,
        advancers=sum(1 for f in vals if f["return_pct"] > 0),
        decliners=sum(1 for f in vals if f["return_pct"] < 0),
        sum_ret=sum(f["return_pct"] for f in vals),
        sum_rs=sum(f["relative_strength_vs_btc"] for f in vals),
        above20=sum(1 for f in vals if f["above_ema20"]),
        above50=sum(1 for f in vals if f["above_ema50"]),
        sum_trend=sum(f["trend_score"] for f in vals),
        sum_atr=sum(f["atr_pct"] for f in vals),
        sum_bbw=sum(f["bb_width"] for f in vals),
        btc=btc_features,
        total_tracked=total_tracked,
    )


def _score(n, advancers, decliners, sum_ret, sum_rs, above20, above50, sum_trend, sum_atr, sum_bbw, btc, total_tracked):
    """live_market_context_accumulator.py:135-204 from the reduced sums."""
    advancers_ratio = advancers / n
    decliners_ratio = decliners / n
    average_return = sum_ret / n
    average_rs = sum_rs / n
    pct_above_ema20 = above20 / n
    pct_above_ema50 = above50 / n
    average_trend_score = sum_trend / n
    average_atr_pct = sum_atr / n
    average_bb_width = sum_bbw / n
    breadth_balance = clamp((advancers_ratio - decliners_ratio) * 1.5)
    ema_balance = clamp(((pct_above_ema20 + pct_above_ema50) - 1.0) * 1.5)
    average_return_score = clamp(average_return * 12.0)
    btc_regime_score = clamp(
        ((btc["return_pct"] * 12.0) + (btc["trend_score"] * 6.0)) if btc is not None else 0.0
    )
    stress_from_volatility = clamp((average_atr_pct - 0.02) * 12.0, 0.0, 1.0)
    stress_from_bandwidth = clamp((average_bb_width - 0.08) * 4.0, 0.0, 1.0)
    stress_from_selloff = clamp((-average_return) * 16.0, 0.0, 1.0)
    market_stress_score = 0.4 * stress_from_volatility + 0.25 * stress_from_bandwidth + 0.35 * stress_from_selloff
    long_tailwind = clamp(
        0.4 * breadth_balance + 0.2 * ema_balance + 0.25 * btc_regime_score + 0.15 * average_return_score
        - 0.35 * market_stress_score
    )
    short_tailwind = clamp(
        -0.35 * breadth_balance - 0.15 * ema_balance - 0.2 * btc_regime_score - 0.15 * average_return_score
        + 0.45 * market_stress_score
    )
    total_tracked = max(total_tracked, n)
    coverage_ratio = n / total_tracked if total_tracked else 0.0
    if n < REQUIRED_FRESH_SYMBOLS or coverage_ratio < MIN_COVERAGE_RATIO:
        return None
    return dict(
        fresh_count=n,
        btc_present=btc is not None,
        total_tracked_symbols=total_tracked,
        coverage_ratio=coverage_ratio,
        advancers=advancers,
        decliners=decliners,
        advancers_ratio=advancers_ratio,
        decliners_ratio=decliners_ratio,
        advancers_decliners_ratio=advancers / max(decliners, 1),
        average_return=average_return,
        average_relative_strength_vs_btc=average_rs,
        pct_above_ema20=pct_above_ema20,
        pct_above_ema50=pct_above_ema50,
        average_trend_score=average_trend_score,
        average_atr_pct=average_atr_pct,
        average_bb_width=average_bb_width,
        btc_return=btc["return_pct"] if btc is not None else 0.0,
        btc_trend_score=btc["trend_score"] if btc is not None else 0.0,
        btc_regime_score=btc_regime_score,
        market_stress_score=market_stress_score,
        long_tailwind=long_tailwind,
        short_tailwind=short_tailwind,
    )


def annotate_market(ctx: dict, prev: dict | None) -> dict:
    """RegimeTransitionDetector._annotate_market_regime (regime_transitions.py:45-160)."""
    breadth_score = clamp((ctx["advancers_ratio"] - 0.5) / 0.25)
    trend_participation = clamp(((ctx["pct_above_ema20"] + ctx["pct_above_ema50"]) - 1.0) * 1.4)
    avg_trend_bias = clamp(ctx["average_trend_score"] * 20.0)
    calm_score = clamp(1.0 - ctx["market_stress_score"], 0.0, 1.0)
    long_score = clamp(
        0.3 * non_negative(ctx["long_tailwind"]) + 0.24 * non_negative(ctx["btc_regime_score"])
        + 0.2 * non_negative(breadth_score) + 0.14 * non_negative(trend_participation) + 0.12 * calm_score,
        0.0,
        1.0,
    )
    short_score = clamp(
        0.28 * non_negative(ctx["short_tailwind"]) + 0.24 * non_negative(-ctx["btc_regime_score"])
        + 0.16 * non_negative(-breadth_score) + 0.1 * non_negative(-avg_trend_bias)
        + 0.22 * ctx["market_stress_score"],
        0.0,
        1.0,
    )
    range_score = clamp(
        0.32 * (1.0 - abs(breadth_score)) + 0.22 * (1.0 - abs(ctx["btc_regime_score"])) + 0.24 * calm_score
        + 0.12 * (1.0 - abs(avg_trend_bias)) + 0.1 * (1.0 - abs(ctx["long_tailwind"] - ctx["short_tailwind"])),
        0.0,
        1.0,
    )
    stress_score = clamp(
        0.7 * ctx["market_stress_score"] + 0.18 * non_negative(-ctx["average_return"] * 20.0)
        + 0.12 * non_negative(short_score - long_score),
        0.0,
        1.0,
    )
    regime = "TRANSITIONAL"
    dominant = max(long_score, short_score, range_score, stress_score)
    if stress_score >= 0.5 and ctx["market_stress_score"] >= 0.35:
        regime = "HIGH_STRESS"
    elif long_score >= 0.44 and long_score >= short_score + 0.08:
        regime = "TREND_UP"
    elif short_score >= 0.42 and short_score >= long_score + 0.08:
        regime = "TREND_DOWN"
    elif range_score >= 0.5:
        regime = "RANGE"
    prev_regime = prev["market_regime"] if prev else None
    transition = None
    strength = 0.0
    transitioning = regime == "TRANSITIONAL"
    if prev is not None and prev_regime is not None and prev_regime != regime:
        transition = market_transition_event(prev_regime, regime)
        prev_scores = (prev["long_regime_score"], prev["short_regime_score"], prev["range_regime_score"], prev["stress_regime_score"])
        cur = (long_score, short_score, range_score, stress_score)
        strength = clamp(dominant + max(abs(a - b) for a, b in zip(cur, prev_scores)) - 0.25, 0.0, 1.0)
        transitioning = transitioning or strength >= 0.08
    out = dict(ctx)
    out.update(
        market_regime=regime,
        previous_market_regime=prev_regime,
        market_regime_transition=transition,
        market_regime_transition_strength=strength,
        long_regime_score=long_score,
        short_regime_score=short_score,
        range_regime_score=range_score,
        stress_regime_score=stress_score,
        regime_is_transitioning=transitioning,
    )
    if prev is None or prev["market_regime"] != regime or prev.get("regime_stable_since") is None:
        out["regime_stable_since"] = ctx.get("timestamp")
    else:
        out["regime_stable_since"] = prev["regime_stable_since"]
    return out


def market_transition_event(prev: str, cur: str) -> str:   # regime_transitions.py:234-249
    if cur == "HIGH_STRESS":
        return "STRESS_SPIKE"
    if prev == "HIGH_STRESS" and cur != "HIGH_STRESS":
        return "STRESS_RELIEF"
    return {"TREND_UP": "ENTERED_TREND_UP", "TREND_DOWN": "ENTERED_TREND_DOWN", "RANGE": "ENTERED_RANGE"}.get(
        cur, "LOST_REGIME_EDGE"
    )


def annotate_symbol(f: dict, prev: dict | None) -> dict:
    """_annotate_symbol_regime (regime_transitions.py:162-232)."""
    ts = f["trend_score"]
    rs = f["relative_strength_vs_btc"]
    up = clamp(0.45 * non_negative(ts * 30.0) + 0.2 * float(f["above_ema20"]) + 0.15 * float(f["above_ema50"])
               + 0.2 * non_negative(rs * 20.0), 0.0, 1.0)
    down = clamp(0.45 * non_negative(-ts * 30.0) + 0.2 * float(not f["above_ema20"]) + 0.15 * float(not f["above_ema50"])
                 + 0.2 * non_negative(-rs * 20.0), 0.0, 1.0)
    rng = clamp(0.38 * (1.0 - min(abs(ts) * 30.0, 1.0)) + 0.34 * (1.0 - min(f["bb_width"] / 0.08, 1.0))
                + 0.28 * (1.0 - min(f["atr_pct"] / 0.04, 1.0)), 0.0, 1.0)
    vol = clamp(0.55 * min(f["atr_pct"] / 0.05, 1.0) + 0.45 * min(f["bb_width"] / 0.12, 1.0), 0.0, 1.0)
    regime = "TRANSITIONAL"
    strength = max(up, down, rng, vol)
    if vol >= 0.72 and abs(f["return_pct"]) >= 0.015:
        regime = "VOLATILE"
    elif up >= 0.52 and up >= down + 0.1:
        regime = "TREND_UP"
    elif down >= 0.52 and down >= up + 0.1:
        regime = "TREND_DOWN"
    elif rng >= 0.5:
        regime = "RANGE"
    prev_regime = prev.get("micro_regime") if prev else None
    transition = None
    tstrength = 0.0
    if prev is not None and prev_regime is not None and prev_regime != regime:
        transition = symbol_transition_event(prev_regime, regime)
        tstrength = clamp(strength + abs(strength - prev["micro_regime_strength"]) - 0.25, 0.0, 1.0)
    out = dict(f)
    out.update(micro_regime=regime, micro_regime_strength=strength, micro_regime_transition=transition,
               micro_regime_transition_strength=tstrength)
    return out


def symbol_transition_event(prev: str, cur: str) -> str:   # regime_transitions.py:251-277
    if cur == "VOLATILE":
        return "VOLATILITY_EXPANSION"
    if prev in {"RANGE", "TRANSITIONAL"} and cur == "TREND_UP":
        return "BREAKOUT_UP"
    if prev in {"RANGE", "TRANSITIONAL"} and cur == "TREND_DOWN":
        return "BREAKDOWN"
    if prev == "TREND_DOWN" and cur == "TREND_UP":
        return "RECOVERY"
    if prev == "TREND_UP" and cur == "RANGE":
        return "MEAN_REVERSION"
    return {"TREND_UP": "ENTERED_TREND_UP", "TREND_DOWN": "ENTERED_TREND_DOWN", "RANGE": "ENTERED_RANGE"}.get(
        cur, "ENTERED_TRANSITIONAL"
    )


def roll_mean_replay(vals, window: int, min_periods: int = 1) -> np.ndarray:
    """pandas 2.3.3 roll_mean for a fixed window, replayed step by step:
    Kahan add / remove with separate compensations, nobs, the same-value run
    (result = the value) and sign (neg_ct) rules of calc_mean. The order of
    floating-point operations is the one bq_store_features replays on the
    device (the restatement is pinned bit-exact against pandas in
    tests/test_oracle_golden.py)."""
    x = np.asarray(vals, dtype=np.float64)
    out = np.empty(x.size)
    s = ca = cr = 0.0
    nobs = neg = same = 0
    prev = x[0] if x.size else 0.0
    for i in range(x.size):
        if i >= window and x[i - window] == x[i - window]:
            v = x[i - window]
            nobs -= 1
            y = -v - cr
            t = s + y
            cr = t - s - y
            s = t
            neg -= 1 if np.signbit(v) else 0
        v = x[i]
        if v == v:
            nobs += 1
            y = v - ca
            t = s + y
            ca = t - s - y
            s = t
            neg += 1 if np.signbit(v) else 0
            same = same + 1 if v == prev else 1
            prev = v
        if nobs >= min_periods and nobs > 0:
            r = s / nobs
            if same >= nobs:
                r = prev
            elif neg == 0 and r < 0:
                r = 0.0
            elif neg == nobs and r > 0:
                r = 0.0
        else:
            r = np.nan
        out[i] = r
    return out


def roll_var_replay(vals, window: int, min_periods: int = 1, ddof: int = 0) -> np.ndarray:
    """pandas 2.3.3 roll_var for a fixed window (compensated Welford add /
    remove, same-value rule -> 0), replayed step by step; see roll_mean_replay."""
    x = np.asarray(vals, dtype=np.float64)
    out = np.empty(x.size)
    nobs = mean = ssq = ca = cr = 0.0
    same = 0
    prev = x[0] if x.size else np.nan
    for i in range(x.size):
        if i >= window and x[i - window] == x[i - window]:
            v = x[i - window]
            nobs -= 1
            if nobs:
                pm = mean - cr
                y = v - cr
                t = y - mean
                cr = t + mean - y
                mean = mean - t / nobs
                ssq = ssq - (v - pm) * (v - mean)
            else:
                mean = ssq = 0.0
        v = x[i]
        if v == v:
            same = same + 1 if v == prev else 1
            prev = v
            nobs += 1
            pm = mean - ca
            y = v - ca
            t = y - mean
            ca = t + mean - y
            mean = mean + t / nobs if nobs else 0.0
            ssq = ssq + (v - pm) * (v - mean)
        if nobs >= min_periods and nobs > ddof:
            r = 0.0 if (nobs == 1 or same >= nobs) else max(ssq / (nobs - ddof), 0.0)
        else:
            r = np.nan
        out[i] = r
    return out
