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

Everything runs through the bq_rolling / bq_ewm kernels plus device tensor
glue in the reference's operation order; there is no CPU path.
"""

from __future__ import annotations

import torch

from . import engine
from .strategies import _clip_lower, _diff, _shift

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


def wilder_rsi(close: torch.Tensor, window: int = 14) -> torch.Tensor:
    """Wilder RSI: ewm(alpha=1/window, min_periods=window, adjust=False) of
    gains/losses, 100*g/(g+l), 50 where g+l == 0 (NaN warm-up kept)."""
    delta = _diff(close, 1)
    gain = _clip_lower(delta, 0.0)
    loss = -torch.where(delta > 0, torch.zeros_like(delta), delta)   # -delta.clip(upper=0), NaN stays
    ag, al = engine.rolling_many(engine.Ewm(gain, alpha=1 / window, min_periods=window),
                                 engine.Ewm(loss, alpha=1 / window, min_periods=window))
    den = ag + al
    return torch.where(den != 0, 100 * ag / den, torch.full_like(den, 50.0))


def trend_score(close: torch.Tensor, fast: int = 20, slow: int = 50) -> torch.Tensor:
    """(ema_fast - ema_slow) / |ema_slow|, 0 where ema_slow == 0."""
    f, s = engine.rolling_many(engine.Ewm(close, span=fast), engine.Ewm(close, span=slow))
    return torch.where(s == 0, torch.zeros_like(s), (f - s) / s.abs())


def adx(high: torch.Tensor, low: torch.Tensor, close: torch.Tensor, window: int = 14) -> torch.Tensor:
    """_compute_adx at every t: rolling-sum DI+/DI-, dx NaN -> 0, mean over
    `window`; NaN (short history) -> 100."""
    hd = _diff(high, 1)
    ld = -_diff(low, 1)
    zero = torch.zeros_like(hd)
    plus_dm = torch.where((hd > ld) & (hd > 0), hd, zero)
    minus_dm = torch.where((ld > hd) & (ld > 0), ld, zero)
    pc = _shift(close, 1)
    tr = torch.fmax(torch.fmax(high - low, (high - pc).abs()), (low - pc).abs())   # max(axis=1) skips NaN
    atr_sum, plus_sum, minus_sum = engine.rolling_many(
        engine.Roll(tr, window, "sum"), engine.Roll(plus_dm, window, "sum"), engine.Roll(minus_dm, window, "sum"))
    plus_di = 100.0 * plus_sum / atr_sum
    minus_di = 100.0 * minus_sum / atr_sum
    total = plus_di + minus_di
    dx = 100.0 * (plus_di - minus_di).abs() / torch.where(total != 0, total, torch.full_like(total, NAN))
    dx = torch.nan_to_num(dx, nan=0.0, posinf=torch.inf, neginf=-torch.inf)   # fillna(0.0)
    a = engine.rolling(dx, window, "mean")
    return torch.where(torch.isnan(a), torch.full_like(a, 100.0), a)


def zscore(close: torch.Tensor, window: int = 20) -> torch.Tensor:
    """_compute_zscore at every t: (c - mean) / std(ddof=0); 0 where std is 0
    or NaN."""
    mean, std = engine.rolling_many(engine.Roll(close, window, "mean"), engine.Roll(close, window, "std0"))
    bad = (std == 0) | torch.isnan(std)
    return torch.where(bad, torch.zeros_like(std), (close - mean) / std)


def top_gainer_features(o, h, l, c, v, qv=None, atr=None, min_history: int = 56, lookback_high: int = 48,
                        volume_window: int = 32, full_extension_bars: int = 96, max_extension: float = 0.50,
                        min_short_extension_cap: float = 0.25):
    """TopGainerEarlyMomentum._features evaluated at every t (prefix frames).
    Returns (values, status): values maps TG_KEYS to [S, T] float64 (NaN where
    status != TG_READY), status is [S, T] int8 (TG_* codes)."""
    S, T = c.shape
    dev = c.device
    eps = 1e-6
    vals: dict[str, torch.Tensor] = {}
    vals["close"], vals["open"], vals["high"], vals["low"], vals["volume"] = c, o, h, l, v
    R, E = engine.Roll, engine.Ewm
    # df["high"].iloc[-49:-1].max(): the 48 highs before t (fewer when short; nan-skipping)
    specs = [R(v, volume_window, "mean"), R(h, lookback_high, "max", min_periods=1, shift=1), E(c, span=20),
             E(c, span=50)]
    if qv is not None:
        specs.append(R(qv, volume_window, "mean"))
    res = engine.rolling_many(*specs)
    vma, vals["previous_high"], e20, e50 = res[:4]
    if qv is not None:
        vals["quote_volume"] = qv
        qvma = res[4]
    else:
        vals["quote_volume"] = v * c
        qvma = vma * c
    t = torch.arange(T, device=dev, dtype=torch.int64)

    def back(k):
        # close.iloc[-k - 1] of the prefix frame (t + 1 rows): index t - k,
        # wrapping like python when t < k (those rows are history_too_short)
        return c[:, torch.remainder(t - k, t + 1)]

    vals["return_1h"] = c / back(4) - 1
    vals["return_2h"] = c / back(8) - 1
    vals["return_6h"] = c / back(24) - 1
    anchor = torch.clamp(t - full_extension_bars, min=0)
    bars = (t - anchor).to(torch.float64)
    vals["extension_return"] = c / c[:, anchor] - 1
    vals["extension_window_bars"] = bars.expand(S, T)
    short_cap = torch.clamp(max_extension * (bars / full_extension_bars), min=min_short_extension_cap)
    cap = torch.where(bars < full_extension_bars, short_cap, torch.full_like(bars, max_extension))
    vals["extension_cap"] = cap.expand(S, T)
    vals["candle_return"] = c / o - 1
    vals["volume_ratio"] = v / (vma + eps)
    vals["quote_volume_ratio"] = vals["quote_volume"] / (qvma + eps)
    rng = h - l
    vals["range_position"] = (c - l) / (rng + eps)
    vals["upper_wick_fraction"] = (h - torch.maximum(o, c)) / (rng + eps)
    vals["ema20"] = e20
    vals["ema50"] = e50
    vals["atr"] = atr if atr is not None else torch.zeros_like(c)
    status = torch.full((S, T), TG_READY, dtype=torch.int8, device=dev)
    finite = torch.ones((S, T), dtype=torch.bool, device=dev)
    for k in TG_KEYS:
        finite &= torch.isfinite(vals[k])
    status[~finite] = TG_NOT_READY
    mn = torch.minimum(torch.minimum(torch.minimum(c, o), torch.minimum(h, l)), v)
    status[~(mn > 0) & ~torch.isnan(mn)] = TG_INVALID_CANDLE   # python min() <= 0
    status[:, : min_history - 1] = TG_SHORT_HISTORY
    ready = status == TG_READY
    out = {k: torch.where(ready, vals[k], torch.full_like(c, NAN)) for k in TG_KEYS}
    return out, status


def mean_reversion_features(o, h, l, c, v, atr, rsi_window: int = 14, volume_ma_window: int = 20,
                            atr_ma_window: int = 20, fast: int = 20, slow: int = 50) -> dict[str, torch.Tensor]:
    """The per-candle inputs MeanReversionFade reads (strategies/mean_reversion_fade.py:240-255):
    rsi / previous_rsi, volume_ma, atr_ma, trend_score and the upper rejection
    ratio of _resolve_entry (:124-134)."""
    rsi = wilder_rsi(c, rsi_window)
    rng = h - l
    vma, ama = engine.rolling_many(engine.Roll(v, volume_ma_window, "mean"), engine.Roll(atr, atr_ma_window, "mean"))
    return {
        "rsi": rsi,
        "previous_rsi": _shift(rsi, 1),
        "volume_ma": vma,
        "atr_ma": ama,
        "trend_score": trend_score(c, fast, slow),
        "upper_rejection_ratio": torch.where(rng > 0, (h - torch.maximum(o, c)) / rng, torch.full_like(c, NAN)),
    }
