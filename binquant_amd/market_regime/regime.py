"""Vectorised market-context scoring and regime annotation (host side).

The device produces, per timestamp, the cross-symbol counts and sums of
``LiveMarketContextAccumulator._build_context``
(market_regime/live_market_context_accumulator.py:135-163) — after an RCCL
all-reduce when symbols are sharded over GPUs. What remains is O(T) scalar
arithmetic, done here with numpy over all timestamps at once:

  * score_contexts      — :96-204 (admission gates, clamp-combined scores)
  * annotate_market     — regime_transitions.py:45-160 (+ transitions, which
                          chain through the previous context: a short loop)
  * annotate_symbols    — regime_transitions.py:162-232, element-wise over
                          [symbols] for one timestamp

All formulas keep the reference's operation order so results agree to a few
ulps; sums arrive in a different (fixed) order than Python's set iteration,
which is why averages are compared with a tolerance and labels exactly away
from their cut points.
"""

from __future__ import annotations

from dataclasses import dataclass, field
from math import ceil

import numpy as np

REQUIRED_FRESH_SYMBOLS = 40   # live_market_context_accumulator.py:13
MIN_COVERAGE_RATIO = 0.70     # :14
TRANSITION_STRENGTH_FLOOR = 0.08   # regime_transitions.py:23

PARTIAL_INDEX = dict(count=0, adv=1, dec=2, above20=3, above50=4, sret=5, strend=6, satr=7, sbbw=8)


def _clamp(x, lo=-1.0, hi=1.0):
    """shared/utils.py:12-13, element-wise (max(lo, min(hi, x)))."""
    return np.maximum(lo, np.minimum(hi, x))


def _nn(x):
    """shared/utils.py:16-17."""
    return np.maximum(0.0, x)


@dataclass
class ContextBatch:
    """Per-timestamp LiveMarketContext fields as arrays ([T]); ``valid[t]`` is
    False where the reference returns None (admission / coverage gates)."""

    timestamp: np.ndarray
    valid: np.ndarray
    fields: dict[str, np.ndarray] = field(default_factory=dict)

    def context_at(self, i: int) -> dict | None:
        if not self.valid[i]:
            return None
        d = {k: (v[i].item() if hasattr(v[i], "item") else v[i]) for k, v in self.fields.items()}
        d["timestamp"] = int(self.timestamp[i])
        return d


def score_contexts(
    partial: np.ndarray,
    btc_return: np.ndarray,
    btc_trend: np.ndarray,
    btc_valid: np.ndarray,
    total_tracked: int,
    fresh_count: np.ndarray | None = None,
    timestamps: np.ndarray | None = None,
) -> ContextBatch:
    """_build_context (:95-242) from reduced partials [T, 10].

    fresh_count[t]: symbols whose last closed candle is t (all of them in a
    [S, T] panel); defaults to total_tracked.
    """
    P = np.asarray(partial, dtype=np.float64)
    T = P.shape[0]
    ix = PARTIAL_INDEX
    n = P[:, ix["count"]]
    fresh = np.full(T, float(total_tracked)) if fresh_count is None else np.asarray(fresh_count, np.float64)
    required = max(REQUIRED_FRESH_SYMBOLS, ceil(total_tracked * MIN_COVERAGE_RATIO))
    with np.errstate(divide="ignore", invalid="ignore"):
        nz = np.where(n > 0, n, np.nan)
        adv, dec = P[:, ix["adv"]], P[:, ix["dec"]]
        advancers_ratio = adv / nz
        decliners_ratio = dec / nz
        advancers_decliners_ratio = adv / np.maximum(dec, 1.0)
        average_return = P[:, ix["sret"]] / nz
        btc_ret = np.where(btc_valid, btc_return, 0.0)
        # sum over symbols of (ret - btc_ret), BTC's own entry 0 (:117-123)
        sum_rs = np.where(btc_valid, P[:, ix["sret"]] - n * btc_ret, 0.0)
        average_rs = sum_rs / nz
        pct_above_ema20 = P[:, ix["above20"]] / nz
        pct_above_ema50 = P[:, ix["above50"]] / nz
        average_trend_score = P[:, ix["strend"]] / nz
        average_atr_pct = P[:, ix["satr"]] / nz
        average_bb_width = P[:, ix["sbbw"]] / nz
    breadth_balance = _clamp((advancers_ratio - decliners_ratio) * 1.5)
    ema_balance = _clamp(((pct_above_ema20 + pct_above_ema50) - 1.0) * 1.5)
    average_return_score = _clamp(average_return * 12.0)
    btc_regime_score = np.where(
        btc_valid, _clamp((btc_return * 12.0) + (btc_trend * 6.0)), 0.0
    )
    stress_from_volatility = _clamp((average_atr_pct - 0.02) * 12.0, 0.0, 1.0)
    stress_from_bandwidth = _clamp((average_bb_width - 0.08) * 4.0, 0.0, 1.0)
    stress_from_selloff = _clamp((-average_return) * 16.0, 0.0, 1.0)
    market_stress_score = 0.4 * stress_from_volatility + 0.25 * stress_from_bandwidth + 0.35 * stress_from_selloff
    long_tailwind = _clamp(
        0.4 * breadth_balance + 0.2 * ema_balance + 0.25 * btc_regime_score + 0.15 * average_return_score
        - 0.35 * market_stress_score
    )
    short_tailwind = _clamp(
        -0.35 * breadth_balance - 0.15 * ema_balance - 0.2 * btc_regime_score - 0.15 * average_return_score
        + 0.45 * market_stress_score
    )
    tracked = np.maximum(float(total_tracked), n)
    coverage_ratio = np.where(tracked > 0, n / np.where(tracked > 0, tracked, 1.0), 0.0)
    valid = (
        (fresh >= required)
        & (total_tracked > 0)
        & (n >= required)
        & (n >= REQUIRED_FRESH_SYMBOLS)
        & (coverage_ratio >= MIN_COVERAGE_RATIO)
    )
    ts = np.arange(T, dtype=np.int64) if timestamps is None else np.asarray(timestamps)
    fields = dict(
        fresh_count=n.astype(np.int64),
        total_tracked_symbols=tracked.astype(np.int64),
        coverage_ratio=coverage_ratio,
        btc_present=np.asarray(btc_valid, bool),
        advancers=adv.astype(np.int64),
        decliners=dec.astype(np.int64),
        advancers_ratio=advancers_ratio,
        decliners_ratio=decliners_ratio,
        advancers_decliners_ratio=advancers_decliners_ratio,
        average_return=average_return,
        average_relative_strength_vs_btc=average_rs,
        pct_above_ema20=pct_above_ema20,
        pct_above_ema50=pct_above_ema50,
        average_trend_score=average_trend_score,
        average_atr_pct=average_atr_pct,
        average_bb_width=average_bb_width,
        btc_return=btc_ret,
        btc_trend_score=np.where(btc_valid, btc_trend, 0.0),
        btc_regime_score=btc_regime_score,
        market_stress_score=market_stress_score,
        long_tailwind=long_tailwind,
        short_tailwind=short_tailwind,
    )
    return ContextBatch(timestamp=ts, valid=valid, fields=fields)


def market_scores(f: dict[str, np.ndarray]) -> dict[str, np.ndarray]:
    """The four regime scores of _annotate_market_regime (regime_transitions.py:50-92)."""
    breadth_score = _clamp((f["advancers_ratio"] - 0.5) / 0.25)
    trend_participation = _clamp(((f["pct_above_ema20"] + f["pct_above_ema50"]) - 1.0) * 1.4)
    avg_trend_bias = _clamp(f["average_trend_score"] * 20.0)
    calm_score = _clamp(1.0 - f["market_stress_score"], 0.0, 1.0)
    long_score = _clamp(
        0.3 * _nn(f["long_tailwind"]) + 0.24 * _nn(f["btc_regime_score"]) + 0.2 * _nn(breadth_score)
        + 0.14 * _nn(trend_participation) + 0.12 * calm_score,
        0.0,
        1.0,
    )
    short_score = _clamp(
        0.28 * _nn(f["short_tailwind"]) + 0.24 * _nn(-f["btc_regime_score"]) + 0.16 * _nn(-breadth_score)
        + 0.1 * _nn(-avg_trend_bias) + 0.22 * f["market_stress_score"],
        0.0,
        1.0,
    )
    range_score = _clamp(
        0.32 * (1.0 - np.abs(breadth_score)) + 0.22 * (1.0 - np.abs(f["btc_regime_score"])) + 0.24 * calm_score
        + 0.12 * (1.0 - np.abs(avg_trend_bias)) + 0.1 * (1.0 - np.abs(f["long_tailwind"] - f["short_tailwind"])),
        0.0,
        1.0,
    )
    stress_score = _clamp(
        0.7 * f["market_stress_score"] + 0.18 * _nn(-f["average_return"] * 20.0) + 0.12 * _nn(short_score - long_score),
        0.0,
        1.0,
    )
    return dict(long=long_score, short=short_score, range=range_score, stress=stress_score)


def classify_market(sc: dict[str, np.ndarray], market_stress: np.ndarray) -> np.ndarray:
    """regime_transitions.py:93-101 (first matching rule wins)."""
    regime = np.full(sc["long"].shape, "TRANSITIONAL", dtype=object)
    high = (sc["stress"] >= 0.5) & (market_stress >= 0.35)
    up = ~high & (sc["long"] >= 0.44) & (sc["long"] >= sc["short"] + 0.08)
    down = ~high & ~up & (sc["short"] >= 0.42) & (sc["short"] >= sc["long"] + 0.08)
    rng = ~high & ~up & ~down & (sc["range"] >= 0.5)
    regime[high] = "HIGH_STRESS"
    regime[up] = "TREND_UP"
    regime[down] = "TREND_DOWN"
    regime[rng] = "RANGE"
    return regime


def market_transition_event(prev: str, cur: str) -> str:
    """regime_transitions.py:234-249."""
    if cur == "HIGH_STRESS":
        return "STRESS_SPIKE"
    if prev == "HIGH_STRESS" and cur != "HIGH_STRESS":
        return "STRESS_RELIEF"
    return {"TREND_UP": "ENTERED_TREND_UP", "TREND_DOWN": "ENTERED_TREND_DOWN", "RANGE": "ENTERED_RANGE"}.get(
        cur, "LOST_REGIME_EDGE"
    )


def annotate_market(batch: ContextBatch, previous: dict | None = None) -> ContextBatch:
    """RegimeTransitionDetector._annotate_market_regime over every valid
    timestamp in order; each context's predecessor is the latest earlier valid
    one (accumulator._get_previous_context, :86-93), seeded by `previous`.

    Vectorised over T: a context depends on its predecessor's regime and four
    scores only, so the predecessor arrays are the valid contexts shifted by
    one (the seed first); `regime_stable_since` is the timestamp of the latest
    run start (a change of regime, or a predecessor without a stable-since)
    carried forward by a running max of the start indices."""
    f = batch.fields
    sc = market_scores(f)
    regime = classify_market(sc, f["market_stress_score"])
    T = len(batch.valid)
    prev_regime = np.full(T, None, dtype=object)
    transition = np.full(T, None, dtype=object)
    strength = np.zeros(T)
    transitioning = regime == "TRANSITIONAL"
    stable_since = np.full(T, None, dtype=object)
    vi = np.flatnonzero(batch.valid)
    n = len(vi)
    if n:
        cur = regime[vi]
        seed_regime = None if previous is None else previous["market_regime"]
        pr = np.empty(n, dtype=object)
        pr[0] = seed_regime
        pr[1:] = cur[:-1]
        if previous is not None:
            prev_regime[vi] = pr
        else:
            prev_regime[vi[1:]] = pr[1:]
        has_prev = np.ones(n, dtype=bool)
        has_prev[0] = previous is not None
        changed = has_prev & np.not_equal(pr, None) & (pr != cur)
        names = ("long", "short", "range", "stress")
        keys = ("long_regime_score", "short_regime_score", "range_regime_score", "stress_regime_score")
        cs = np.stack([sc[k][vi] for k in names])          # [4, n]
        ps = np.empty_like(cs)
        ps[:, 1:] = cs[:, :-1]
        ps[:, 0] = [previous[k] for k in keys] if changed[0] else 0.0
        ci = np.flatnonzero(changed)
        if len(ci):
            dominant = cs[:, ci].max(axis=0)
            delta = np.abs(cs[:, ci] - ps[:, ci]).max(axis=0)
            st = np.fmin(1.0, np.fmax(0.0, (dominant + delta) - 0.25))   # Python min(1, max(0, x))
            idx = vi[ci]
            strength[idx] = st
            transitioning[idx] = transitioning[idx] | (st >= TRANSITION_STRENGTH_FLOOR)
            transition[idx] = [market_transition_event(a, b) for a, b in zip(pr[ci], cur[ci])]
        # run starts: no predecessor, a different regime, or a predecessor without stable-since
        start = ~has_prev | (pr != cur)
        carried = None
        if not start[0]:
            carried = previous.get("regime_stable_since")
            start[0] = carried is None
        ts = batch.timestamp[vi]
        last = np.maximum.accumulate(np.where(start, np.arange(n), -1))
        ss = np.empty(n, dtype=object)
        ok = last >= 0
        ss[ok] = np.asarray(ts[last[ok]], dtype=np.int64).astype(object)   # Python ints, as int(ts)
        ss[~ok] = carried   # a seed run continuing from `previous`
        stable_since[vi] = ss
    f.update(
        market_regime=regime,
        previous_market_regime=prev_regime,
        market_regime_transition=transition,
        market_regime_transition_strength=strength,
        long_regime_score=sc["long"],
        short_regime_score=sc["short"],
        range_regime_score=sc["range"],
        stress_regime_score=sc["stress"],
        regime_is_transitioning=transitioning,
        regime_stable_since=stable_since,
    )
    return batch


def annotate_symbols(
    trend_score, above_ema20, above_ema50, relative_strength, bb_width, atr_pct, return_pct,
    prev_regime=None, prev_strength=None,
) -> dict[str, np.ndarray]:
    """_annotate_symbol_regime (regime_transitions.py:162-232) element-wise
    over symbols (and optionally their previous micro regime)."""
    ts = np.asarray(trend_score, np.float64)
    a20 = np.asarray(above_ema20, np.float64)
    a50 = np.asarray(above_ema50, np.float64)
    rs = np.asarray(relative_strength, np.float64)
    bbw = np.asarray(bb_width, np.float64)
    atr = np.asarray(atr_pct, np.float64)
    up = _clamp(0.45 * _nn(ts * 30.0) + 0.2 * a20 + 0.15 * a50 + 0.2 * _nn(rs * 20.0), 0.0, 1.0)
    down = _clamp(0.45 * _nn(-ts * 30.0) + 0.2 * (1.0 - a20) + 0.15 * (1.0 - a50) + 0.2 * _nn(-rs * 20.0), 0.0, 1.0)
    rng = _clamp(
        0.38 * (1.0 - np.minimum(np.abs(ts) * 30.0, 1.0)) + 0.34 * (1.0 - np.minimum(bbw / 0.08, 1.0))
        + 0.28 * (1.0 - np.minimum(atr / 0.04, 1.0)),
        0.0,
        1.0,
    )
    vol = _clamp(0.55 * np.minimum(atr / 0.05, 1.0) + 0.45 * np.minimum(bbw / 0.12, 1.0), 0.0, 1.0)
    strength = np.maximum(np.maximum(up, down), np.maximum(rng, vol))
    regime = np.full(ts.shape, "TRANSITIONAL", dtype=object)
    v = (vol >= 0.72) & (np.abs(np.asarray(return_pct, np.float64)) >= 0.015)
    u = ~v & (up >= 0.52) & (up >= down + 0.1)
    d = ~v & ~u & (down >= 0.52) & (down >= up + 0.1)
    r = ~v & ~u & ~d & (rng >= 0.5)
    regime[v] = "VOLATILE"
    regime[u] = "TREND_UP"
    regime[d] = "TREND_DOWN"
    regime[r] = "RANGE"
    out = dict(micro_regime=regime, micro_regime_strength=strength)
    if prev_regime is not None:
        trans = np.full(ts.shape, None, dtype=object)
        tstr = np.zeros(ts.shape)
        prev_regime = np.asarray(prev_regime, dtype=object)
        changed = np.array([p is not None for p in prev_regime], dtype=bool) & (prev_regime != regime)
        for i in np.flatnonzero(changed):
            trans[i] = symbol_transition_event(prev_regime[i], regime[i])
            tstr[i] = min(1.0, max(0.0, strength[i] + abs(strength[i] - prev_strength[i]) - 0.25))
        out.update(micro_regime_transition=trans, micro_regime_transition_strength=tstr)
    return out


def symbol_transition_event(prev: str, cur: str) -> str:
    """regime_transitions.py:251-277."""
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
