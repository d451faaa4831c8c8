"""Batched inline indicator helpers of the signal generators.

The reference's strategies compute a handful of small indicators inline on one
symbol's frame and read the last row(s). Here every helper evaluates the whole
[S, T] panel on the device, so column t is what the reference returns for the
prefix frame df.iloc[:t + 1]:

* wilder_rsi         MeanReversionFade._rsi (strategies/mean_reversion_fade.py:88-109)
* trend_score        MeanReversionFade._trend_score (:149-155), also the EMA9/21
                     trend of strategies/coinrule/price_tracker.py:204-211
* ema                close.ewm(span, adjust=False, min_periods) as used by
                     price_tracker.py:204-205, top_gainer_early_momentum.py:153-154,
                     gradual_gainer_retest.py:257-259 (read at t-1),
                     coinrule/buy_the_dip.py:63-71 (min_periods=1)
* adx, zscore        RangeBbRsiMeanReversion._compute_adx / _compute_zscore
                     (strategies/range_bb_rsi_mean_reversion.py:101-138)
* top_gainer_features TopGainerEarlyMomentum._features
                     (strategies/top_gainer_early_momentum.py:92-160)
* mean_reversion_features  the entry inputs of MeanReversionFade (:240-255)

wilder_rsi, zscore and adx default to the time-parallel kernels of
bq_signals.hip (one launch each, 1e-9 of pandas); exact=True runs the
replay composition instead — the bq_rolling / bq_ewm kernels plus fused
element-wise programs (binquant_amd.fused) in the reference's operation
order, equal to pandas bit for bit. The other helpers use that composition.
Rows with missing candles (NaN) keep pandas' NaN rules on the fast kernels
too (bq_signals.hip: z-score / ADX re-sum the windows a gap touched; the
Wilder RSI row is replayed with pandas' own ewm update from the first gap).
There is no CPU path.
"""

from __future__ import annotations

import torch

from . import engine
from . import fused as F

NAN = float("nan")

# TopGainerEarlyMomentum._features status strings, as int8 codes
TG_READY, TG_SHORT_HISTORY, TG_INVALID_CANDLE, TG_NOT_READY = 0, 1, 2, 3
TG_STATUS = {TG_READY: "features_ready", TG_SHORT_HISTORY: "history_too_short",
             TG_INVALID_CANDLE: "invalid_candle_values", TG_NOT_READY: "indicators_not_ready"}
TG_KEYS = ("close", "open", "high", "low", "volume", "quote_volume", "previous_high", "return_1h", "return_2h",
           "return_6h", "extension_return", "extension_window_bars", "extension_cap", "candle_return",
           "volume_ratio", "quote_volume_ratio", "range_position", "upper_wick_fraction", "ema20", "ema50", "atr")


def ema(close: torch.Tensor, span: int, min_periods: int = 0) -> torch.Tensor:
    """close.ewm(span=span, adjust=False, min_periods=min_periods).mean()."""
    return engine.ewm(close, span=span, min_periods=min_periods)


def _rsi_ex(close: torch.Tensor, window: int) -> F.Ex:
    C = F.inp(close)
    delta = F.diff(C, 1)
    g = F.run({"g": F.clip_lower(delta, 0.0), "l": -F.where(delta > 0, 0.0, delta)})   # -delta.clip(upper=0)
    ag, al = engine.rolling_many(engine.Ewm(g["g"], alpha=1 / window, min_periods=window),
                                 engine.Ewm(g["l"], alpha=1 / window, min_periods=window))
    AG = F.inp(ag)
    den = AG + al
    return F.where(den != 0, 100 * AG / den, 50.0)


def wilder_rsi(close: torch.Tensor, window: int = 14, exact: bool = False) -> torch.Tensor:
    """Wilder RSI: ewm(alpha=1/window, min_periods=window, adjust=False) of
    gains/losses, 100*g/(g+l), 50 where g+l == 0 (NaN warm-up kept)."""
    if not exact:
        return engine.wilder_rsi(close, window)
    return F.run({"rsi": _rsi_ex(close, window)})["rsi"]


def _trend_ex(close: torch.Tensor, fast: int, slow: int) -> F.Ex:
    f, s = engine.rolling_many(engine.Ewm(close, span=fast), engine.Ewm(close, span=slow))
    Fx, Sx = F.inp(f), F.inp(s)
    return F.where(Sx == 0, 0.0, (Fx - Sx) / Sx.abs())


def trend_score(close: torch.Tensor, fast: int = 20, slow: int = 50) -> torch.Tensor:
    """(ema_fast - ema_slow) / |ema_slow|, 0 where ema_slow == 0."""
    return F.run({"t": _trend_ex(close, fast, slow)})["t"]


def adx(high: torch.Tensor, low: torch.Tensor, close: torch.Tensor, window: int = 14,
        exact: bool = False) -> torch.Tensor:
    """_compute_adx at every t: rolling-sum DI+/DI-, dx NaN -> 0, mean over
    `window`; NaN (short history) -> 100."""
    if not exact and window <= 64:
        return engine.adx(high, low, close, window)
    H, L, C = F.inp(high), F.inp(low), F.inp(close)
    hd = F.diff(H, 1)
    ld = -F.diff(L, 1)
    pc = F.shift(C, 1)
    dm = F.run({
        "tr": F.fmax(F.fmax(H - L, (H - pc).abs()), (L - pc).abs()),   # max(axis=1) skips NaN
        "plus": F.where((hd > ld) & (hd > 0), hd, 0.0),
        "minus": F.where((ld > hd) & (ld > 0), ld, 0.0),
    })
    atr_sum, plus_sum, minus_sum = engine.rolling_many(
        engine.Roll(dm["tr"], window, "sum"), engine.Roll(dm["plus"], window, "sum"),
        engine.Roll(dm["minus"], window, "sum"))
    A = F.inp(atr_sum)
    plus_di = 100.0 * F.inp(plus_sum) / A
    minus_di = 100.0 * F.inp(minus_sum) / A
    total = plus_di + minus_di
    dx = 100.0 * (plus_di - minus_di).abs() / F.where(total != 0, total, NAN)
    dx = F.run({"dx": F.fillna(dx, 0.0)})["dx"]
    a = engine.rolling(dx, window, "mean")
    return F.run({"adx": F.fillna(a, 100.0)})["adx"]


def zscore(close: torch.Tensor, window: int = 20, exact: bool = False) -> torch.Tensor:
    """_compute_zscore at every t: (c - mean) / std(ddof=0); 0 where std is 0
    or NaN."""
    if not exact:
        return engine.zscore(close, window)
    mean, std = engine.rolling_many(engine.Roll(close, window, "mean"), engine.Roll(close, window, "std0"))
    SD = F.inp(std)
    bad = (SD == 0) | F.isnan(SD)
    return F.run({"z": F.where(bad, 0.0, (F.inp(close) - mean) / SD)})["z"]


def top_gainer_features(o, h, l, c, v, qv=None, atr=None, min_history: int = 56, lookback_high: int = 48,
                        volume_window: int = 32, full_extension_bars: int = 96, max_extension: float = 0.50,
                        min_short_extension_cap: float = 0.25):
    """TopGainerEarlyMomentum._features evaluated at every t (prefix frames).
    Returns (values, status): values maps TG_KEYS to [S, T] float64 (NaN where
    status != TG_READY), status is [S, T] int8 (TG_* codes)."""
    S, T = c.shape
    dev = c.device
    eps = 1e-6
    R, E = engine.Roll, engine.Ewm
    # df["high"].iloc[-49:-1].max(): the 48 highs before t (fewer when short; nan-skipping)
    specs = [R(v, volume_window, "mean"), R(h, lookback_high, "max", min_periods=1, shift=1), E(c, span=20),
             E(c, span=50)]
    if qv is not None:
        specs.append(R(qv, volume_window, "mean"))
    res = engine.rolling_many(*specs)
    vma, prev_high, e20, e50 = res[:4]
    qvma = res[4] if qv is not None else None
    C, O, H, L, V = (F.inp(x) for x in (c, o, h, l, v))
    QV = F.inp(qv) if qv is not None else V * C
    QVMA = F.inp(qvma) if qv is not None else F.inp(vma) * C
    # close.iloc[-k - 1] of the prefix frame (t + 1 rows) is close[t - k]; rows
    # with t < k are history_too_short (min_history > 24), masked below
    t = torch.arange(T, device=dev, dtype=torch.int64)
    anchor = torch.clamp(t - full_extension_bars, min=0)
    bars = (t - anchor).to(torch.float64)
    short_cap = torch.clamp(max_extension * (bars / full_extension_bars), min=min_short_extension_cap)
    cap = torch.where(bars < full_extension_bars, short_cap, torch.full_like(bars, max_extension))
    BARS, CAP = F.inp(bars), F.inp(cap)
    # close at the anchor: close[t - 96], or the first close while t < 96
    c_anchor = F.where(BARS < full_extension_bars, F.inp(c[:, :1]), F.shift(C, full_extension_bars))
    rng = H - L
    ex = {
        "close": C, "open": O, "high": H, "low": L, "volume": V, "quote_volume": QV,
        "previous_high": F.inp(prev_high),
        "return_1h": C / F.shift(C, 4) - 1,
        "return_2h": C / F.shift(C, 8) - 1,
        "return_6h": C / F.shift(C, 24) - 1,
        "extension_return": C / c_anchor - 1,
        "extension_window_bars": BARS,
        "extension_cap": CAP,
        "candle_return": C / O - 1,
        "volume_ratio": V / (F.inp(vma) + eps),
        "quote_volume_ratio": QV / (QVMA + eps),
        "range_position": (C - L) / (rng + eps),
        "upper_wick_fraction": (H - F.maximum(O, C)) / (rng + eps),
        "ema20": F.inp(e20),
        "ema50": F.inp(e50),
        "atr": F.inp(atr) if atr is not None else F.const(0.0),
    }
    # status: not finite -> NOT_READY, then python min() <= 0 -> INVALID, then short history
    finite = None
    for k in TG_KEYS:
        x = ex[k]
        ok = ~F.isnan(x - x)          # x - x is NaN for NaN and +-inf
        finite = ok if finite is None else finite & ok
    mn = F.minimum(F.minimum(F.minimum(C, O), F.minimum(H, L)), V)
    invalid = ~(mn > 0) & ~F.isnan(mn)
    short = F.inp(t.to(torch.float64)) < float(min_history - 1)   # len(prefix) = t + 1 < min_history
    code = F.where(short, float(TG_SHORT_HISTORY),
                   F.where(invalid, float(TG_INVALID_CANDLE), F.where(finite, float(TG_READY), float(TG_NOT_READY))))
    status_f = F.run({"status": code}, S, T)["status"]
    ready = F.inp(status_f) == float(TG_READY)
    out = F.run({k: F.where(ready, ex[k], NAN) for k in TG_KEYS}, S, T)
    return out, status_f.to(torch.int8)


_LEADERSHIP_FUSED = True   # False: the staged pipeline for every parameter set (tests)


def gradual_gainer_leadership(open_time: torch.Tensor, close: torch.Tensor, btc_time: torch.Tensor,
                              btc_close: torch.Tensor, rs_quantile: float = 0.80, rs_lookback: int = 96,
                              min_history: int = 100, min_count: int = 20, short: int = 8, long: int = 24):
    """GradualGainerRetest._leadership_allows at every t (column t = the
    method on the prefix frame df.iloc[:t + 1]; strategies/gradual_gainer_retest.py
    :131-196), against the benchmark frame (btc_time ascending, duplicates:
    the later row wins, as the reference's dict does).

    * btc close at each candle's open_time: the left merge bq_align;
    * _relative_strengths: all of the last short·3+1 = 25 times present in the
      benchmark and every close > 0 (a rolling(25) integer sum of that flag),
      rs_2h / rs_6h = c/c[-8] - b/b[-8], c/c[-24] - b/b[-24];
    * the history: one entry per position i >= 24 of the last 96 whose times i,
      i-8, i-24 are all in the benchmark with the six closes > 0 — NaN
      elsewhere, so the 80th-percentile threshold sorted(h)[int((n-1) q)] is
      rolling(96, min_periods=20).quantile(q, interpolation="lower")
      (bq_rolling_batch, BQ_ROLL_QLOWER; order statistics by bit selection);
    * leader = rs_2h > 0 and rs_6h > 0 and rs >= threshold for both.

    Returns {"leader": bool [S, T], "rs_2h": [S, T], "rs_6h": [S, T]} with the
    method's fall-backs: (False, 0.0, 0.0) when the strengths are None or the
    frame is shorter than min_history, (False, rs_2h, rs_6h) when fewer than
    min_count history entries exist.

    The strategy's lookback runs in one pass (engine.leadership,
    bq_leadership); any others run the staged pipeline below. A NaN close is
    not > 0 here, so it never enters the history or the strengths; the
    reference's Python min(...) skips a NaN unless it is its first argument
    (:148, :178) and can append NaN strengths, whose place in sorted() is
    undefined: frames with missing closes are parity-unpinned (the golden
    frames hold none; pre_process drops such rows before the strategies)."""
    fused = engine.leadership(open_time, close, btc_time, btc_close, rs_quantile, rs_lookback, min_history,
                              min_count, short, long) if _LEADERSHIP_FUSED else None
    if fused is not None:   # the strategy's lookback: one pass (bq_leadership)
        return fused
    # any other parameters: the staged pipeline
    S, T = close.shape
    recent = long + 1
    b = engine.align(open_time, btc_time, btc_close)
    C, B = F.inp(close), F.inp(b)
    pos = ((C > 0) & (F.shift(C, short) > 0) & (F.shift(C, long) > 0)
           & (B > 0) & (F.shift(B, short) > 0) & (F.shift(B, long) > 0))
    rs2 = C / F.shift(C, short) - B / F.shift(B, short)
    rs6 = C / F.shift(C, long) - B / F.shift(B, long)
    st = F.run({"h2": F.where(pos, rs2, NAN), "h6": F.where(pos, rs6, NAN),
                "ok": F.where((C > 0) & (B > 0), 1.0, 0.0), "rs2": rs2, "rs6": rs6}, S, T)
    R = engine.Roll
    thr2, thr6, okn = engine.rolling_many(
        R(st["h2"], rs_lookback, "qlower", q=rs_quantile, min_periods=min_count),
        R(st["h6"], rs_lookback, "qlower", q=rs_quantile, min_periods=min_count),
        R(st["ok"], recent, "isum", min_periods=recent))
    n = torch.arange(1, T + 1, device=close.device, dtype=torch.float64)
    R2, R6, T2, T6 = F.inp(st["rs2"]), F.inp(st["rs6"]), F.inp(thr2), F.inp(thr6)
    strengths = (F.inp(okn) == float(recent)) & (F.inp(n) >= float(min_history))
    leader = strengths & ~F.isnan(T2) & (R2 > 0) & (R6 > 0) & (R2 >= T2) & (R6 >= T6)
    res = F.run({"leader": leader, "rs_2h": F.where(strengths, R2, 0.0), "rs_6h": F.where(strengths, R6, 0.0)}, S, T)
    return res


def mean_reversion_features(o, h, l, c, v, atr, rsi_window: int = 14, volume_ma_window: int = 20,
                            atr_ma_window: int = 20, fast: int = 20, slow: int = 50) -> dict[str, torch.Tensor]:
    """The per-candle inputs MeanReversionFade reads (strategies/mean_reversion_fade.py:240-255):
    rsi / previous_rsi, volume_ma, atr_ma, trend_score and the upper rejection
    ratio of _resolve_entry (:124-134)."""
    rsi = _rsi_ex(c, rsi_window)
    vma, ama = engine.rolling_many(engine.Roll(v, volume_ma_window, "mean"), engine.Roll(atr, atr_ma_window, "mean"))
    H, L, O, C = F.inp(h), F.inp(l), F.inp(o), F.inp(c)
    rng = H - L
    res = F.run({
        "rsi": rsi,
        "previous_rsi": F.shift(rsi, 1),
        "trend_score": _trend_ex(c, fast, slow),
        "upper_rejection_ratio": F.where(rng > 0, (H - F.maximum(O, C)) / rng, NAN),
    })
    return {"rsi": res["rsi"], "previous_rsi": res["previous_rsi"], "volume_ma": vma, "atr_ma": ama,
            "trend_score": res["trend_score"], "upper_rejection_ratio": res["upper_rejection_ratio"]}
