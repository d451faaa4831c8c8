"""Direct per-candle pins of the headline enrich columns against the
reference's own in-repo twins (tests/golden/headline_twins.npz, written by
tests/golden/make_golden.py --only twins from the real functions on every
prefix frame). pybinbot — the library behind the headline columns — is absent
(uv.lock:1391-1403); these twins are the reference code that computes the same
quantities:

  ema20 / ema50 (spans 20 / 50)  LiveMarketContextAccumulator._compute_symbol_features
                                 (market_regime/live_market_context_accumulator.py:266-267)
  ATR (rolling-14 TR mean)       the same function's atr_pct = atr / close (:256-268, 284)
  bb_upper / bb_mid / bb_lower   its bb_width = (upper - lower) / |mid| with ddof 0,
  (window 20, ddof 0, k 2)       k = 2 (:269-272, 286-290)
  ema spans 9 / 21               MeanReversionFade._trend_score run with its EMA windows
                                 set to 9 / 21: the expression of
                                 strategies/coinrule/price_tracker.py:204-205
  ema spans 20 / 50 (again)      MeanReversionFade._trend_score (mean_reversion_fade.py:150-155)
  rsi (SMA, windows 14 and 6)    BBExtremeReversion._compute_rsi
                                 (strategies/coinrule/bb_extreme_reversion.py:134-150)

Compared where the enrich column is defined (its rolling windows use
min_periods = window; the twins use min_periods = 1 for ATR / BB): a window
holding a missing candle is NaN in enrich and must be one that holds a NaN.
Tolerances (tests/util.py): rtol 1e-9 with the absolute floor 1e-11 x scale
(the frame's mean |close| for the EMAs, 1 for the dimensionless ratios
atr_pct / bb_width / trend score, 100 for RSI). exact=True (the oracle, which
runs pandas' own ewm) asks the EMAs and trend scores to be bit-equal; the
panel kernel's EMA scan carries differ from pandas' serial recursion by ulps
(DESIGN §4.1), so it is held to the bar — the tick path is the bit-exact one
(tests/test_tick_gpu.py)."""

from __future__ import annotations

from pathlib import Path

import numpy as np

GOLDEN = Path(__file__).resolve().parent / "golden" / "headline_twins.npz"
RTOL, ATOL_REL = 1e-9, 1e-11

# IndicatorParams of the two enrich runs (as keyword dicts: engine.IndicatorParams
# and the oracle's parameter dict take the same names)
PARAMS_A = dict(ema_spans=(20, 50), atr_window=14, bb_window=20, bb_ddof=0, bb_k=2.0, rsi_window=14)
PARAMS_B = dict(ema_spans=(9, 21), rsi_window=6, bb_ddof=0)


def load():
    d = np.load(GOLDEN)
    names = [str(n) for n in d["names"]]
    fcols = [str(c) for c in d["feature_columns"]]
    frames = {}
    for n in names:
        fr = {k: d[f"{n}__{k}"] for k in ("open", "high", "low", "close", "volume")}
        fr["features"] = {c: d[f"{n}__features"][:, i] for i, c in enumerate(fcols)}
        for k in ("sma_rsi14", "sma_rsi6", "trend_9_21", "trend_20_50"):
            fr[k] = d[f"{n}__{k}"]
        frames[n] = fr
    return frames


def _trend(fast, slow):
    """MeanReversionFade._trend_score's arithmetic on the enrich EMA columns."""
    out = np.empty_like(fast)
    for t in range(fast.size):
        out[t] = 0.0 if slow[t] == 0 else float((fast[t] - slow[t]) / abs(slow[t]))
    return out


def _close(got, want, scale, name):
    err = np.abs(got - want)
    lim = RTOL * np.abs(want) + ATOL_REL * scale
    bad = ~(err <= lim)
    assert not bad.any(), (f"{name}: {int(bad.sum())} of {got.size} beyond the bar, first at "
                           f"{int(np.argmax(bad))}: got {got[bad][0]!r} want {want[bad][0]!r}")


def _window_has_nan(x, w):
    """For each t: x[t - w + 1 .. t] holds a NaN or starts before 0."""
    bad = np.isnan(x).astype(np.int64)
    cs = np.r_[0, np.cumsum(bad)]
    t = np.arange(x.size)
    lo = t - w + 1
    return (lo < 0) | (cs[t + 1] - cs[np.maximum(lo, 0)] > 0)


def _same(got, want, scale, name, exact):
    assert np.array_equal(np.isnan(got), np.isnan(want)), f"{name}: NaN pattern differs"
    m = ~np.isnan(want)
    if exact:
        assert np.array_equal(got[m], want[m]), f"{name}: {int((got[m] != want[m]).sum())} candles differ"
    else:
        _close(got[m], want[m], scale, name)


def check_frame(name, fr, a, b, exact=False):
    """a / b: the 14 enrich columns of the frame with PARAMS_A / PARAMS_B
    (1-D arrays). Returns the number of candles compared per pin."""
    c, h, l = fr["close"], fr["high"], fr["low"]
    n = c.size
    f = fr["features"]
    have = ~np.isnan(f["ema20"])   # the function returned features (k >= 2)
    price = float(np.nanmean(np.abs(c)))
    counts = {}
    # EMA family: pandas' ewm recursion
    for col in ("ema20", "ema50"):
        _same(a[col][have], f[col][have], price, f"{name} {col}", exact)
        counts[col] = int(have.sum())
    ts = _trend(a["ema20"], a["ema50"])
    _same(ts[have], f["trend_score"][have], 1.0, f"{name} trend_score (20/50)", exact)
    _same(ts, fr["trend_20_50"], 1.0, f"{name} _trend_score 20/50", exact)
    ts9 = _trend(b["ema20"], b["ema50"])   # the PARAMS_B spans are (9, 21)
    _same(ts9, fr["trend_9_21"], 1.0, f"{name} _trend_score 9/21", exact)
    counts["ema9_21"] = n
    # ATR: rolling-14 mean of the true range, read through atr_pct = atr / close
    tr = np.fmax(h - l, np.fmax(np.abs(h - np.r_[np.nan, c[:-1]]), np.abs(l - np.r_[np.nan, c[:-1]])))
    atr = a["ATR"]
    defined = ~np.isnan(atr)
    assert not (defined & _window_has_nan(tr, 14)).any(), f"{name} ATR: a value over a window with a gap"
    m = defined & have & (c != 0)
    _close(atr[m] / c[m], f["atr_pct"][m], 1.0, f"{name} ATR (atr_pct)")
    counts["ATR"] = int(m.sum())
    # Bollinger, ddof 0, k 2: bb_width = (upper - lower) / |mid|
    mid, up, lo = a["bb_mid"], a["bb_upper"], a["bb_lower"]
    defined = ~np.isnan(mid)
    assert not (defined & _window_has_nan(c, 20)).any(), f"{name} bb: a value over a window with a gap"
    m = defined & have & (mid != 0)
    _close((up[m] - lo[m]) / np.abs(mid[m]), f["bb_width"][m], 1.0, f"{name} bb_width")
    counts["bb"] = int(m.sum())
    # SMA RSI: the helper needs window + 1 closes (None -> NaN: flat windows too)
    for cols, w, key in ((a, 14, "sma_rsi14"), (b, 6, "sma_rsi6")):
        got, want = cols["rsi"][w:], fr[key][w:]
        assert np.array_equal(np.isnan(got), np.isnan(want)), \
            f"{name} rsi{w}: NaN pattern differs at {np.argwhere(np.isnan(got) != np.isnan(want))[:5].ravel() + w}"
        m = ~np.isnan(want)
        _close(got[m], want[m], 100.0, f"{name} rsi{w}")
        counts[key] = int(m.sum())
    return counts
