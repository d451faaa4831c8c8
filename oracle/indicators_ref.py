"""pandas restatement of the pybinbot.Indicators contract used by binquant.

TEST INFRASTRUCTURE ONLY (see oracle/__init__.py). pybinbot==1.11.8 is not
available offline; each formula below is the assumption the GPU kernels are
held to, with the reference call site / in-repo twin it follows.

Call sites: producers/context_evaluator.py:249-261 (indicators_enrichment),
strategies/coinrule/price_tracker.py:185 (mfi).
"""

from __future__ import annotations

import numpy as np
import pandas as pd

DEFAULTS = dict(
    ma_periods=(7, 25, 100),
    macd_fast=12,
    macd_slow=26,
    macd_signal=9,
    rsi_window=14,
    bb_window=20,
    bb_ddof=1,
    bb_k=2.0,
    atr_window=14,
    twap_window=12,
    ema_spans=(20, 50),
    mfi_window=14,
)


def moving_averages(df: pd.DataFrame, period: int) -> pd.DataFrame:
    """ma_{period} = close.rolling(period).mean()  (context_evaluator.py:249-251;
    post_process then drops the warm-up NaNs, :435-441)."""
    df[f"ma_{period}"] = df["close"].rolling(period).mean()
    return df


def macd(df: pd.DataFrame, fast: int = 12, slow: int = 26, signal: int = 9) -> pd.DataFrame:
    """macd = EMA12 - EMA26 (adjust=False); macd_signal = EMA9(macd).
    Called at context_evaluator.py:254; read at price_tracker.py:184 and
    gradual_gainer_retest.py:328. macd_signal: parity unpinned."""
    close = df["close"]
    e_fast = close.ewm(span=fast, adjust=False).mean()
    e_slow = close.ewm(span=slow, adjust=False).mean()
    df["macd"] = e_fast - e_slow
    df["macd_signal"] = df["macd"].ewm(span=signal, adjust=False).mean()
    return df


def rsi(df: pd.DataFrame, window: int = 14) -> pd.DataFrame:
    """SMA-smoothed RSI: the pybinbot column 'uses a simple rolling mean'
    (strategies/mean_reversion_fade.py:42-44); formula of the in-repo twin
    strategies/coinrule/bb_extreme_reversion.py:134-150."""
    delta = df["close"].astype(float).diff()
    gain = delta.where(delta > 0, 0.0).rolling(window).mean()
    loss = (-delta.where(delta < 0, 0.0)).rolling(window).mean()
    rs = gain / loss
    df["rsi"] = 100 - (100 / (1 + rs))
    return df


def ma_spreads(df: pd.DataFrame) -> pd.DataFrame:
    """No in-repo reader. Restated as the spreads of the MAs
    (percent): parity unpinned."""
    df["big_ma_spread"] = (abs(df["ma_100"] - df["ma_25"]) / df["ma_100"]) * 100
    df["small_ma_spread"] = (abs(df["ma_25"] - df["ma_7"]) / df["ma_25"]) * 100
    return df


def bollinguer_spreads(
    df: pd.DataFrame, window: int = 20, num_std: float = 2.0, ddof: int = 1
) -> pd.DataFrame:
    """bb_mid/bb_upper/bb_lower (context_evaluator.py:202-204 readers).
    Window 20, k=2; ddof=1 is pandas' default std (the in-repo twin at
    live_market_context_accumulator.py:270 uses ddof=0)."""
    mid = df["close"].rolling(window).mean()
    std = df["close"].rolling(window).std(ddof=ddof)
    df["bb_mid"] = mid
    df["bb_upper"] = mid + (num_std * std)
    df["bb_lower"] = mid - (num_std * std)
    return df


def set_twap(df: pd.DataFrame, periods: int = 12) -> pd.DataFrame:
    """twap = rolling mean of the bar price (open+high+low+close)/4 over
    `periods` bars (reader: strategies/coinrule/coinrule.py:67). Parity
    unpinned."""
    bar = (df["open"] + df["high"] + df["low"] + df["close"]) / 4
    df["twap"] = bar.rolling(periods).mean()
    return df


def true_range(df: pd.DataFrame) -> pd.Series:
    """TR with skip-NaN max: first row is high-low
    (live_market_context_accumulator.py:256-264)."""
    prev = df["close"].shift(1)
    return pd.concat(
        [df["high"] - df["low"], (df["high"] - prev).abs(), (df["low"] - prev).abs()],
        axis=1,
    ).max(axis=1)


def atr(df: pd.DataFrame, window: int = 14) -> pd.DataFrame:
    """ATR = TR.rolling(window).mean() — the rolling-mean smoothing of the
    in-repo twin live_market_context_accumulator.py:268 (mean_reversion_fade.py:45
    says the shared ATR 'matches the backtest'). Smoothing choice: parity unpinned."""
    df["ATR"] = true_range(df).rolling(window).mean()
    return df


def mfi_series(df: pd.DataFrame, window: int = 14) -> pd.Series:
    """Money-flow index column (typical price, positive/negative flow sums)."""
    tp = (df["high"] + df["low"] + df["close"]) / 3
    mf = tp * df["volume"]
    prev = tp.shift(1)
    pos = mf.where(tp > prev, 0.0).rolling(window).sum()
    neg = mf.where(tp < prev, 0.0).rolling(window).sum()
    return 100 - (100 / (1 + pos / neg))


def mfi(df: pd.DataFrame, window: int = 14) -> float:
    """Indicators.mfi(df) -> float of the last bar (price_tracker.py:185)."""
    return float(mfi_series(df, window).iloc[-1])


def ema(df: pd.DataFrame, span: int) -> pd.Series:
    """close.ewm(span, adjust=False).mean() (live_market_context_accumulator.py:266-267)."""
    return df["close"].ewm(span=span, adjust=False).mean()


def indicators_enrichment(df: pd.DataFrame, p: dict | None = None) -> pd.DataFrame:
    """ContextEvaluator.indicators_enrichment (producers/context_evaluator.py:240-263)
    plus the mfi / ema20 / ema50 columns of the canonical 14-column set."""
    p = {**DEFAULTS, **(p or {})}
    for period in p["ma_periods"]:
        df = moving_averages(df, period)
    df = macd(df, p["macd_fast"], p["macd_slow"], p["macd_signal"])
    df = rsi(df, p["rsi_window"])
    df = bollinguer_spreads(df, p["bb_window"], p["bb_k"], p["bb_ddof"])
    df = set_twap(df, p["twap_window"])
    df = atr(df, p["atr_window"])
    df[f"ema{p['ema_spans'][0]}"] = ema(df, p["ema_spans"][0])
    df[f"ema{p['ema_spans'][1]}"] = ema(df, p["ema_spans"][1])
    df["mfi"] = mfi_series(df, p["mfi_window"])
    return df


CANONICAL = (
    "ma_7",
    "ma_25",
    "ma_100",
    "macd",
    "macd_signal",
    "rsi",
    "bb_upper",
    "bb_mid",
    "bb_lower",
    "ATR",
    "twap",
    "ema20",
    "ema50",
    "mfi",
)


def enrich_panel(o, h, l, c, v, p: dict | None = None) -> dict[str, np.ndarray]:
    """Per-symbol reference call pattern over a [S][T] panel: one pandas frame
    per symbol, exactly as the reference processes one symbol per message."""
    o, h, l, c, v = (np.asarray(x, dtype=np.float64) for x in (o, h, l, c, v))
    S, T = c.shape
    out = {k: np.empty((S, T)) for k in CANONICAL}
    for s in range(S):
        df = pd.DataFrame({"open": o[s], "high": h[s], "low": l[s], "close": c[s], "volume": v[s]})
        df = indicators_enrichment(df, p)
        for k in CANONICAL:
            out[k][s] = df[k].to_numpy()
    return out


def ema_family_panel(c, p: dict | None = None) -> dict[str, np.ndarray]:
    """The EMA-family columns (macd, macd_signal, ema20, ema50) of
    indicators_enrichment for every row of a [S, T] close panel at once:
    DataFrame.ewm runs pandas' ewm recursion column by column over a [T, S]
    frame — the same Cython routine as the per-frame Series calls of macd()
    and ema() above — so each row equals enrich_panel's bit for bit, at a
    fraction of the per-symbol cost (the C3 10k-symbol checks)."""
    p = {**DEFAULTS, **(p or {})}
    close = pd.DataFrame(np.asarray(c, dtype=np.float64).T)
    e_fast = close.ewm(span=p["macd_fast"], adjust=False).mean()
    e_slow = close.ewm(span=p["macd_slow"], adjust=False).mean()
    m = e_fast - e_slow
    sig = m.ewm(span=p["macd_signal"], adjust=False).mean()
    out = {"macd": m, "macd_signal": sig,
           f"ema{p['ema_spans'][0]}": close.ewm(span=p["ema_spans"][0], adjust=False).mean(),
           f"ema{p['ema_spans'][1]}": close.ewm(span=p["ema_spans"][1], adjust=False).mean()}
    return {k: np.ascontiguousarray(v.to_numpy().T) for k, v in out.items()}


def tick_frame_rows(o, h, l, c, v, t: int, frame: int = 400, p: dict | None = None) -> dict[str, np.ndarray]:
    """What the reference computes per closed-kline message at candle t: it
    re-fetches the last KlinesProvider.LIMIT = 400 candles
    (consumers/klines_provider.py:40,201-215) and runs indicators_enrichment on
    that frame (producers/context_evaluator.py:367-371); the value it reads is
    the frame's last row. frame = 0: the whole history [0, t]."""
    a = 0 if frame == 0 else max(0, t - frame + 1)
    sl = slice(a, t + 1)
    got = enrich_panel(*(np.asarray(x)[:, sl] for x in (o, h, l, c, v)), p)
    return {k: x[:, -1] for k, x in got.items()}


def ema_family_frame(c, t: int, frame: int = 400, p: dict | None = None) -> dict[str, np.ndarray]:
    """ema_family_panel over each row's frame [t - frame + 1, t] (the
    reference's per-message frame, see tick_frame_rows), last column: equal
    bit for bit to tick_frame_rows' EMA family, for every row of a wide panel."""
    a = 0 if frame == 0 else max(0, t - frame + 1)
    got = ema_family_panel(np.asarray(c)[:, a : t + 1], p)
    return {k: x[:, -1] for k, x in got.items()}


def ewm_scalar(x, alpha: float) -> np.ndarray:
    """Pure-Python restatement of pandas' ewm(adjust=False, ignore_na=False)
    mean recursion (pandas/_libs/window/aggregations.pyx `ewm`), used to pin the
    update formula the GPU replay uses; small inputs only."""
    x = np.asarray(x, dtype=np.float64)
    out = np.empty_like(x)
    if x.size == 0:
        return out
    om = 1.0 - alpha
    weighted = x[0]
    out[0] = weighted
    old_wt = 1.0
    for i in range(1, x.size):
        cur = x[i]
        is_obs = cur == cur
        if weighted == weighted:
            if is_obs:
                old_wt *= om
                if weighted != cur:
                    weighted = old_wt * weighted + alpha * cur
                    weighted /= old_wt + alpha
                old_wt = 1.0
            else:
                old_wt *= om
        elif is_obs:
            weighted = cur
        out[i] = weighted
    return out


def pct_change_pad(x, periods: int = 96) -> np.ndarray:
    """Series.pct_change(periods) under pandas 2.3.3's default
    fill_method='pad' (the BTC 24h change, producers/context_evaluator.py:
    427-430): forward-fill, then f / f.shift(periods) - 1. numpy restatement
    (leading NaNs stay NaN), pinned to tests/golden/btc_change.npz."""
    x = np.asarray(x, dtype=np.float64)
    idx = np.where(np.isnan(x), -1, np.arange(x.size))
    idx = np.maximum.accumulate(idx) if x.size else idx
    f = np.where(idx >= 0, x[np.maximum(idx, 0)], np.nan)
    out = np.full_like(f, np.nan)
    if periods < f.size:
        with np.errstate(divide="ignore", invalid="ignore"):
            out[periods:] = f[periods:] / f[:-periods] - 1
    return out


def beta_corr_series(close, btc_close, window: int = 50) -> tuple[np.ndarray, np.ndarray]:
    """ContextEvaluator.dynamic_btc_beta_corr (producers/context_evaluator.py:154-194)
    evaluated at every candle t of an index-aligned pair: the raw (unrounded)
    beta/corr of the last row of the prefix [0, t]; NaN while fewer than
    `window` returns exist."""
    alt = pd.Series(np.log(np.asarray(close, float) / np.roll(np.asarray(close, float), 1)))
    btc = pd.Series(np.log(np.asarray(btc_close, float) / np.roll(np.asarray(btc_close, float), 1)))
    alt.iloc[0] = np.nan
    btc.iloc[0] = np.nan
    r = pd.concat([alt, btc], axis=1, keys=["alt", "btc"]).dropna()
    cov = r["alt"].rolling(window).cov(r["btc"])
    var = r["btc"].rolling(window).var()
    beta = (cov / var.replace(0, np.nan)).reindex(range(len(alt))).to_numpy()
    corr = r["alt"].rolling(window).corr(r["btc"]).reindex(range(len(alt))).to_numpy()
    return beta, corr


def dynamic_btc_beta_corr(close, btc_close, window: int = 50) -> tuple[float, float]:
    """Scalar form at the last row, with the reference's NaN -> 0 mapping and
    the (0, 0) short-history case (rounding is pybinbot's round_numbers: not applied)."""
    if len(close) - 1 < window:
        return 0.0, 0.0
    b, c = beta_corr_series(close, btc_close, window)
    return (0.0 if np.isnan(b[-1]) else float(b[-1])), (0.0 if np.isnan(c[-1]) else float(c[-1]))


def supertrend(df: pd.DataFrame, multiplier: float = 3.0, period: int = 10) -> pd.DataFrame:
    """pybinbot Indicators.set_supertrend(df, multiplier=3.0) as called at
    strategies/coinrule/coinrule.py:143 ("period adjusted to 10"); the
    consumer reads bool(df["supertrend"].iloc[-1]) (:160). pybinbot is absent:
    this is the common band-recursion form (parity unpinned). hl2 = (h+l)/2,
    ATR = the `atr` restatement above, bands hl2 +- m*ATR; for t >= 1 the
    trend flips up when close > upper[t-1], down when close < lower[t-1],
    otherwise it holds and the band on the trend's side ratchets."""
    hl2 = (df["high"] + df["low"]) / 2
    a = true_range(df).rolling(period).mean()
    upper = (hl2 + (multiplier * a)).to_numpy(np.float64).copy()
    lower = (hl2 - (multiplier * a)).to_numpy(np.float64).copy()
    close = df["close"].to_numpy(np.float64)
    up = np.ones(len(df), dtype=bool)
    for t in range(1, len(df)):
        p = t - 1
        if close[t] > upper[p]:
            up[t] = True
        elif close[t] < lower[p]:
            up[t] = False
        else:
            up[t] = up[p]
            if up[t] and lower[t] < lower[p]:
                lower[t] = lower[p]
            if not up[t] and upper[t] > upper[p]:
                upper[t] = upper[p]
    df["supertrend"] = up
    df["supertrend_upper"] = upper
    df["supertrend_lower"] = lower
    return df


def exact_zscore(window_closes) -> float:
    """RangeBbRsiMeanReversion._compute_zscore (strategies/range_bb_rsi_mean_reversion.py:132-138)
    of the last close against its window, in exact rational arithmetic (mean
    and ddof-0 variance exact, one sqrt and one division in float64). pandas'
    online roll_var drifts from this by up to ~1e-6 relative in windows that
    are nearly constant (e.g. one candle off a flat run: z = sqrt(w - 1));
    the parity tests use it to show such a deviation is pandas' rounding."""
    from fractions import Fraction
    from math import sqrt

    w = [Fraction(float(v)) for v in np.asarray(window_closes, dtype=np.float64)]
    m = sum(w) / len(w)
    var = sum((v - m) ** 2 for v in w) / len(w)
    if var == 0:
        return 0.0
    return float(w[-1] - m) / sqrt(float(var))


def exact_std(window, ddof: int = 1) -> float:
    """x.rolling(w).std(ddof) of a full window in exact rational arithmetic
    (mean and variance exact, one sqrt in float64). pandas' online roll_var
    drifts from this where the std is small against the values; the spike
    pass's two-pass std (bq_spike_base_std) is held to it there
    (tests/util.assert_close_or_exact)."""
    from fractions import Fraction
    from math import sqrt

    w = [Fraction(float(v)) for v in np.asarray(window, dtype=np.float64)]
    if len(w) <= ddof:
        return float("nan")
    m = sum(w) / len(w)
    var = sum((v - m) ** 2 for v in w) / (len(w) - ddof)
    return sqrt(float(var))


def gradual_gainer_leadership(open_time, close, btc_time, btc_close, q: float = 0.80, lookback: int = 96,
                              min_history: int = 100, min_count: int = 20, short: int = 8, long: int = 24):
    """GradualGainerRetest._leadership_allows (strategies/gradual_gainer_retest.py:131-196)
    at every prefix t of each row, vectorised with pandas: the benchmark
    close by open_time (a dict in the reference: the later of duplicated
    times wins), the history entry at i needs times i, i-8, i-24 present and
    the six closes > 0, threshold = sorted(history)[int((len - 1) * q)] over
    the last `lookback` positions (rolling quantile, interpolation "lower"),
    the strengths need the last 25 times present and every close > 0.
    Returns (leader bool [S, T], rs_2h, rs_6h) with the method's fall-backs."""
    open_time = np.asarray(open_time, dtype=np.int64)
    close = np.asarray(close, dtype=np.float64)
    S, T = close.shape
    bmap = pd.Series(np.asarray(btc_close, float), index=np.asarray(btc_time, np.int64))
    bmap = bmap[~bmap.index.duplicated(keep="last")]
    lead = np.zeros((S, T), dtype=bool)
    r2o, r6o = np.zeros((S, T)), np.zeros((S, T))
    for s in range(S):
        c = pd.Series(close[s])
        b = pd.Series(bmap.reindex(open_time[s]).to_numpy())
        pos = ((c > 0) & (c.shift(short) > 0) & (c.shift(long) > 0) & (b > 0) & (b.shift(short) > 0)
               & (b.shift(long) > 0))
        rs2 = c / c.shift(short) - b / b.shift(short)
        rs6 = c / c.shift(long) - b / b.shift(long)
        h2, h6 = rs2.where(pos), rs6.where(pos)
        t2 = h2.rolling(lookback, min_periods=min_count).quantile(q, interpolation="lower")
        t6 = h6.rolling(lookback, min_periods=min_count).quantile(q, interpolation="lower")
        ok = ((c > 0) & (b > 0)).astype(float).rolling(long + 1).sum() == long + 1
        strengths = ok.to_numpy() & (np.arange(1, T + 1) >= min_history)
        lead[s] = strengths & t2.notna().to_numpy() & (rs2 > 0).to_numpy() & (rs6 > 0).to_numpy() \
            & (rs2 >= t2).to_numpy() & (rs6 >= t6).to_numpy()
        r2o[s] = np.where(strengths, rs2.to_numpy(), 0.0)
        r6o[s] = np.where(strengths, rs6.to_numpy(), 0.0)
    return lead, r2o, r6o
