"""pybinbot.Indicators-compatible DataFrame API backed by the gfx950 kernels.

Drop-in for the calls binquant makes (producers/context_evaluator.py:249-261,
strategies/coinrule/price_tracker.py:185):

    df = Indicators.moving_averages(df, 7)       # adds "ma_7"
    df = Indicators.macd(df=df)                  # "macd", "macd_signal"
    df = Indicators.rsi(df=df)                   # "rsi"
    df = Indicators.ma_spreads(df)               # "big_ma_spread", "small_ma_spread"
    df = Indicators.bollinguer_spreads(df)       # "bb_upper", "bb_mid", "bb_lower"
    df = Indicators.set_twap(df)                 # "twap"
    df = Indicators.atr(df=df, window=14)        # "ATR"
    df = Indicators.set_supertrend(df, 3.0)      # "supertrend" (+ final bands)
    value = Indicators.mfi(df, window=14)        # float of the last candle

Each call returns the frame with the columns added (callers rebind, as in the
reference). ``indicators_enrichment(df)`` runs the whole
ContextEvaluator.indicators_enrichment set in ONE launch, and
``Indicators.batch(panel)`` / ``enrich_frames(frames)`` process many symbols
per launch — the batched form the hot path is meant to use. Frames of
different lengths are end-padded into one [S, T_max] panel: every output at t
depends only on candles <= t, so padding never changes a valid row.

Inputs are coerced with pd.to_numeric like Candles.pre_process does; a missing
OHLCV column raises ValueError naming it (tests/test_ohlc.py:35-64 semantics).
"""

from __future__ import annotations

from collections.abc import Mapping, Sequence

import numpy as np
import pandas as pd
import torch

from . import engine
from ._lib import ENRICH_COLUMNS, INPUT_FIELDS, MAX_WINDOW

_DEVICE = "cuda"


def _device() -> torch.device:
    if not torch.cuda.is_available():
        raise RuntimeError("binquant_amd.Indicators needs a HIP device (no CPU fallback)")
    return torch.device(_DEVICE)


def _column(df: pd.DataFrame, name: str) -> np.ndarray:
    if name not in df.columns:
        if name == "volume":
            return np.zeros(len(df))
        if name == "open":
            name = "close"
        else:
            raise ValueError(f"Missing required candle field '{name}'.")
    vals = pd.to_numeric(df[name], errors="coerce").to_numpy(dtype=np.float64)
    return vals


def _frame_inputs(df: pd.DataFrame) -> list[np.ndarray]:
    if "close" not in df.columns:
        raise ValueError("Missing required candle field 'close'.")
    return [_column(df, f) for f in INPUT_FIELDS]


def _run(df: pd.DataFrame, params: engine.IndicatorParams, columns) -> dict[str, np.ndarray]:
    host = _frame_inputs(df)   # validates columns before touching the device
    dev = _device()
    ins = [torch.from_numpy(np.ascontiguousarray(x)).to(dev)[None, :] for x in host]
    out = engine.enrich(*ins, params=params, columns=columns)
    return {k: v[0].cpu().numpy() for k, v in out.items()}


def _check_window(w: int, what: str) -> int:
    w = int(w)
    if not 1 <= w <= MAX_WINDOW:
        raise ValueError(f"{what}: window {w} outside [1, {MAX_WINDOW}]")
    return w


class Indicators:
    """Static-method surface of pybinbot.Indicators (names and arguments as
    called in binquant). Each method mutates and returns the frame."""

    @staticmethod
    def moving_averages(df: pd.DataFrame, period: int = 7) -> pd.DataFrame:
        p = engine.IndicatorParams(ma_periods=(_check_window(period, "moving_averages"), 25, 100))
        df[f"ma_{int(period)}"] = _run(df, p, ("ma_7",))["ma_7"]
        return df

    @staticmethod
    def macd(df: pd.DataFrame, fast: int = 12, slow: int = 26, signal: int = 9) -> pd.DataFrame:
        p = engine.IndicatorParams(macd_fast=fast, macd_slow=slow, macd_signal=signal)
        r = _run(df, p, ("macd", "macd_signal"))
        df["macd"] = r["macd"]
        df["macd_signal"] = r["macd_signal"]
        return df

    @staticmethod
    def rsi(df: pd.DataFrame, window: int = 14) -> pd.DataFrame:
        p = engine.IndicatorParams(rsi_window=_check_window(window, "rsi"))
        df["rsi"] = _run(df, p, ("rsi",))["rsi"]
        return df

    @staticmethod
    def ma_spreads(df: pd.DataFrame) -> pd.DataFrame:
        """Spreads of the moving averages (percent). No in-repo reader
        (SURVEY §8a a4); needs ma_7/ma_25/ma_100, computed if absent."""
        for p in (7, 25, 100):
            if f"ma_{p}" not in df.columns:
                Indicators.moving_averages(df, p)
        df["big_ma_spread"] = (abs(df["ma_100"] - df["ma_25"]) / df["ma_100"]) * 100
        df["small_ma_spread"] = (abs(df["ma_25"] - df["ma_7"]) / df["ma_25"]) * 100
        return df

    @staticmethod
    def bollinguer_spreads(df: pd.DataFrame, window: int = 20, num_std: float = 2.0, ddof: int = 1) -> pd.DataFrame:
        p = engine.IndicatorParams(bb_window=_check_window(window, "bollinguer_spreads"), bb_k=num_std, bb_ddof=ddof)
        r = _run(df, p, ("bb_upper", "bb_mid", "bb_lower"))
        df["bb_mid"] = r["bb_mid"]
        df["bb_upper"] = r["bb_upper"]
        df["bb_lower"] = r["bb_lower"]
        return df

    @staticmethod
    def set_twap(df: pd.DataFrame, periods: int = 12) -> pd.DataFrame:
        p = engine.IndicatorParams(twap_window=_check_window(periods, "set_twap"))
        df["twap"] = _run(df, p, ("twap",))["twap"]
        return df

    @staticmethod
    def atr(df: pd.DataFrame, window: int = 14) -> pd.DataFrame:
        p = engine.IndicatorParams(atr_window=_check_window(window, "atr"))
        df["ATR"] = _run(df, p, ("ATR",))["ATR"]
        return df

    @staticmethod
    def mfi(df: pd.DataFrame, window: int = 14) -> float:
        p = engine.IndicatorParams(mfi_window=_check_window(window, "mfi"))
        return float(_run(df, p, ("mfi",))["mfi"][-1])

    @staticmethod
    def set_supertrend(df: pd.DataFrame, multiplier: float = 3.0, period: int = 10) -> pd.DataFrame:
        """Adds "supertrend" (bool: uptrend) and the final bands
        "supertrend_upper" / "supertrend_lower" (coinrule.py:143-160 reads
        bool(df["supertrend"].iloc[-1]))."""
        period = _check_window(period, "set_supertrend")
        host = _frame_inputs(df)
        dev = _device()
        h, l, c = (torch.from_numpy(np.ascontiguousarray(x)).to(dev)[None, :] for x in host[1:4])
        r = engine.supertrend(h, l, c, period=period, multiplier=float(multiplier), exact=True)
        for k, v in r.items():
            df[k] = v[0].cpu().numpy()
        return df

    @staticmethod
    def batch(panel: Mapping[str, np.ndarray | torch.Tensor], params: engine.IndicatorParams | None = None,
              columns=ENRICH_COLUMNS) -> dict[str, torch.Tensor]:
        """[S, T] panel (numpy or device tensors) -> {column: [S, T] device tensor}."""
        dev = _device()
        ins = []
        for f in INPUT_FIELDS:
            x = panel[f]
            if not isinstance(x, torch.Tensor):
                x = torch.from_numpy(np.ascontiguousarray(np.asarray(x, dtype=np.float64)))
            ins.append(x.to(dev, dtype=torch.float64))
        return engine.enrich(*ins, params=params, columns=columns)


def indicators_enrichment(df: pd.DataFrame, params: engine.IndicatorParams | None = None) -> pd.DataFrame:
    """ContextEvaluator.indicators_enrichment (producers/context_evaluator.py:240-263)
    in one kernel launch: ma_7/25/100, macd (+macd_signal), rsi, ma spreads,
    bb_upper/bb_mid/bb_lower, twap, ATR — plus ema20/ema50 and mfi."""
    r = _run(df, params or engine.IndicatorParams(), ENRICH_COLUMNS)
    for k in ENRICH_COLUMNS:
        df[k] = r[k]
    df["big_ma_spread"] = (abs(df["ma_100"] - df["ma_25"]) / df["ma_100"]) * 100
    df["small_ma_spread"] = (abs(df["ma_25"] - df["ma_7"]) / df["ma_25"]) * 100
    return df


def enrich_frames(frames: Sequence[pd.DataFrame], params: engine.IndicatorParams | None = None,
                  columns=ENRICH_COLUMNS) -> list[pd.DataFrame]:
    """Enrich many symbols' frames (ragged lengths allowed) in ONE launch."""
    if not frames:
        return []
    lens = [len(f) for f in frames]
    T = max(lens)
    S = len(frames)
    host = {f: np.zeros((S, T)) for f in INPUT_FIELDS}
    for s, df in enumerate(frames):
        vals = _frame_inputs(df)
        n = lens[s]
        for f, v in zip(INPUT_FIELDS, vals):
            host[f][s, :n] = v
            if n and n < T:
                host[f][s, n:] = v[-1]   # end padding (never read by valid rows)
    out = Indicators.batch(host, params=params, columns=columns)
    host_out = {k: v.cpu().numpy() for k, v in out.items()}
    res = []
    for s, df in enumerate(frames):
        n = lens[s]
        for k in columns:
            df[k] = host_out[k][s, :n]
        res.append(df)
    return res


def dynamic_btc_beta_corr(df: pd.DataFrame, df_btc: pd.DataFrame, window: int = 50,
                          decimals: int | None = 6) -> tuple[float, float]:
    """Drop-in for ContextEvaluator.dynamic_btc_beta_corr
    (producers/context_evaluator.py:154-194): the frames are inner-joined on the
    index on the host (as the reference does), the rolling beta/corr run on the
    GPU (bq_beta_corr). Returns (0, 0) below `window` aligned returns and maps
    NaN to 0; values are rounded to `decimals` with Python's round() in place
    of pybinbot.round_numbers (decimals=None: unrounded)."""
    joined = pd.DataFrame({"alt": pd.to_numeric(df["close"], errors="coerce")}).join(
        pd.DataFrame({"btc": pd.to_numeric(df_btc["close"], errors="coerce")}), how="inner"
    )
    if len(joined) - 1 < window:
        return 0.0, 0.0
    dev = _device()
    c = torch.from_numpy(joined["alt"].to_numpy(np.float64)).to(dev)[None, :]
    b = torch.from_numpy(joined["btc"].to_numpy(np.float64)).to(dev)
    out = engine.beta_corr(c, b, window=window)
    beta = float(out["beta"][0, -1])
    corr = float(out["corr"][0, -1])
    beta = 0.0 if np.isnan(beta) else beta
    corr = 0.0 if np.isnan(corr) else corr
    if decimals is not None:
        beta, corr = round(beta, decimals), round(corr, decimals)
    return beta, corr


def dynamic_btc_beta_corr_frames(frames: Sequence[pd.DataFrame], df_btc: pd.DataFrame, window: int = 50,
                                 decimals: int | None = 6, key: str = "open_time") -> list[tuple[float, float]]:
    """Batched dynamic_btc_beta_corr for many symbols' frames against one
    benchmark frame, joined on the `key` timestamp column (the frames' time
    index): per-frame log returns, inner join, dropna (bq_join_returns), then
    rolling(window) beta/corr at each symbol's last joined row
    (bq_beta_corr_pairs). (0, 0) below `window` joined returns; NaN -> 0."""
    if not frames:
        return []
    dev = _device()
    S = len(frames)
    lens = [len(f) for f in frames]
    T = max(1, max(lens))
    ts = np.zeros((S, T), dtype=np.int64)
    cl = np.full((S, T), np.nan)
    for s, df in enumerate(frames):
        n = lens[s]
        if n:
            ts[s, :n] = pd.to_numeric(df[key]).to_numpy(np.int64)
            ts[s, n:] = ts[s, n - 1]
            cl[s, :n] = pd.to_numeric(df["close"], errors="coerce").to_numpy(np.float64)
    bts_h = pd.to_numeric(df_btc[key]).to_numpy(np.int64)
    bts = torch.from_numpy(bts_h).to(dev)
    bcl = torch.from_numpy(pd.to_numeric(df_btc["close"], errors="coerce").to_numpy(np.float64)).to(dev)
    # pairs per row: each candle t >= 1 joins every benchmark row holding its
    # time (pandas' many-to-many inner join), so the exact bound is the sum of
    # those multiplicities — known here on the host, no device round trip
    cap = T
    if bts_h.size:
        for s, n_s in enumerate(lens):
            if n_s > 1:
                k = ts[s, 1:n_s]
                cap = max(cap, int((np.searchsorted(bts_h, k, "right") - np.searchsorted(bts_h, k, "left")).sum()))
    x, y, n = engine.join_returns(torch.from_numpy(ts).to(dev), torch.from_numpy(cl).to(dev), bts, bcl, lens=lens,
                                  capacity=cap)
    bc = engine.beta_corr_pairs(x, y, window=window)
    n = n.cpu().numpy()
    last = torch.from_numpy(np.maximum(n - 1, 0)).to(dev)
    rows = torch.arange(S, device=dev)
    beta = bc["beta"][rows, last].cpu().numpy()
    corr = bc["corr"][rows, last].cpu().numpy()
    res = []
    for s in range(S):
        if n[s] < window:
            res.append((0.0, 0.0))
            continue
        b = 0.0 if np.isnan(beta[s]) else float(beta[s])
        c = 0.0 if np.isnan(corr[s]) else float(corr[s])
        if decimals is not None:
            b, c = round(b, decimals), round(c, decimals)
        res.append((b, c))
    return res


def btc_price_change(df_btc: pd.DataFrame, periods: int = 96) -> float:
    """BTC 24h change of ContextEvaluator.process_data (producers/context_evaluator.py:427-430):
    close.pct_change(periods=96) * 100 at the last row, with pandas 2.3.3's
    default pad fill (a missing close takes the previous one, at the last row
    and at t - 96 alike, reaching as far back as the frame goes), on the device
    (engine.pct_change over the whole column); NaN when the frame is too short
    or no close precedes t - 96, as pandas."""
    c = pd.to_numeric(df_btc["close"], errors="coerce").to_numpy(np.float64)
    if len(c) <= periods:
        return float("nan")
    x = torch.from_numpy(np.ascontiguousarray(c)).to(_device())[None, :]
    return float(engine.pct_change(x, periods)[0, -1] * 100)
