"""pybinbot.Candles-compatible frame preparation.

Mirrors the calls binquant makes (producers/context_evaluator.py:364-433,
tests/test_ohlc.py):

    raw = Candles(exchange=ExchangeId.BINANCE, candles=rows)
    df = raw.pre_process()              # rows -> typed frame (ensure_ohlc)
    df = indicators_enrichment(df)
    df = raw.post_process(df)           # drop warm-up NaN rows
    df_1h = raw.resample(df_15m, interval="1h")   # on the GPU (bq_resample)

pybinbot is absent; behaviour pinned by the reference's own
tests/test_ohlc.py (missing columns named in one ValueError, string columns
coerced to numbers, an all-NaN quote_asset_volume rejected). The rest —
Binance/KuCoin row layouts, sort + de-duplication by open_time (keep last,
as market_state_store.py:30-38 does for the store), post_process = dropna +
fresh index, resample aggregations (open first, high max, low min, close
last, volumes/trades sum, close_time last) — is the restatement, parity
unpinned against pybinbot. ``resample`` and ``resample_frames`` run on the
device; there is no CPU path.
"""

from __future__ import annotations

import re
from collections.abc import Sequence

import numpy as np
import pandas as pd
import torch

from . import engine

KLINE_COLUMNS = (
    "open_time",
    "open",
    "high",
    "low",
    "close",
    "volume",
    "close_time",
    "quote_asset_volume",
    "number_of_trades",
    "taker_buy_base_asset_volume",
    "taker_buy_quote_asset_volume",
)
# tests/test_ohlc.py:35-43: dropping volume + close_time must name both
REQUIRED_COLUMNS = ("open_time", "open", "high", "low", "close", "volume", "close_time")
# columns that may not be entirely non-numeric (tests/test_ohlc.py:59-64)
NON_EMPTY_COLUMNS = REQUIRED_COLUMNS + ("quote_asset_volume",)
# KuCoin REST klines: [time (s), open, close, high, low, volume, turnover]
KUCOIN_COLUMNS = ("open_time", "open", "close", "high", "low", "volume", "quote_asset_volume")

RESAMPLE_AGG = {
    "open": "first",
    "high": "max",
    "low": "min",
    "close": "last",
    "volume": "sum",
    "close_time": "last",
    "quote_asset_volume": "sum",
    "number_of_trades": "sum",
    "taker_buy_base_asset_volume": "sum",
    "taker_buy_quote_asset_volume": "sum",
}

_UNIT_MS = {"s": 1_000, "m": 60_000, "min": 60_000, "h": 3_600_000, "d": 86_400_000, "w": 604_800_000}


def interval_ms(interval: str | int) -> int:
    """"15m" / "1h" / "4h" / "1d" (pandas offset aliases "15min", "1H" too) -> ms."""
    if isinstance(interval, (int, np.integer)):
        return int(interval)
    m = re.fullmatch(r"\s*(\d*)\s*([a-zA-Z]+)\s*", str(interval))
    if not m or m.group(2).lower() not in _UNIT_MS:
        raise ValueError(f"unsupported interval {interval!r}")
    return int(m.group(1) or 1) * _UNIT_MS[m.group(2).lower()]


def _exchange_name(exchange) -> str:
    v = getattr(exchange, "value", exchange)
    return str(v or "binance").lower()


class Candles:
    """Row -> frame preparation for one symbol's klines (pybinbot.Candles surface)."""

    def __init__(self, exchange=None, candles=None):
        self.exchange = exchange
        self.candles = candles if candles is not None else []

    # -- validation ---------------------------------------------------------
    def ensure_ohlc(self, df: pd.DataFrame) -> pd.DataFrame:
        missing = [c for c in REQUIRED_COLUMNS if c not in df.columns]
        if missing:
            raise ValueError(f"Missing required kline columns: {', '.join(missing)}")
        df = df.copy()
        for c in KLINE_COLUMNS:
            if c in df.columns:
                df[c] = pd.to_numeric(df[c], errors="coerce")
        if len(df):
            empty = [c for c in NON_EMPTY_COLUMNS if c in df.columns and df[c].isna().all()]
            if empty:
                raise ValueError(f"Kline columns with no numeric values: {', '.join(empty)}")
        for c in ("open_time", "close_time"):
            if df[c].notna().all():
                df[c] = df[c].astype("int64")
        return df

    # -- rows -> frame --------------------------------------------------------
    def _frame(self) -> pd.DataFrame:
        rows = self.candles
        if isinstance(rows, pd.DataFrame):
            return rows.copy()
        if len(rows) == 0:
            return pd.DataFrame(columns=list(KLINE_COLUMNS))
        if isinstance(rows[0], dict):
            return pd.DataFrame(list(rows))
        if _exchange_name(self.exchange) == "kucoin":
            df = pd.DataFrame([list(r)[: len(KUCOIN_COLUMNS)] for r in rows], columns=list(KUCOIN_COLUMNS))
            df["open_time"] = pd.to_numeric(df["open_time"], errors="coerce") * 1000
            return df
        width = len(KLINE_COLUMNS)
        return pd.DataFrame([list(r)[:width] for r in rows], columns=list(KLINE_COLUMNS[: len(rows[0][:width])]))

    def pre_process(self) -> pd.DataFrame:
        df = self._frame()
        if df.empty:
            return df
        if "close_time" not in df.columns and "open_time" in df.columns and len(df) > 1:
            step = pd.to_numeric(df["open_time"], errors="coerce").diff().median()
            df["close_time"] = pd.to_numeric(df["open_time"], errors="coerce") + step - 1
        df = self.ensure_ohlc(df)
        df = df.sort_values("open_time", kind="stable").drop_duplicates("open_time", keep="last")
        return df.reset_index(drop=True)

    def post_process(self, df: pd.DataFrame) -> pd.DataFrame:
        df = df.dropna()
        return df.reset_index(drop=True)

    # -- resampling (device) ----------------------------------------------------
    def resample(self, df: pd.DataFrame, interval: str | int = "1h") -> pd.DataFrame:
        return resample_frames([df], interval)[0]


def _device() -> torch.device:
    if not torch.cuda.is_available():
        raise RuntimeError("binquant_amd.Candles.resample needs a HIP device (no CPU fallback)")
    return torch.device("cuda")


def resample_frames(frames: Sequence[pd.DataFrame], interval: str | int = "1h") -> list[pd.DataFrame]:
    """Resample many symbols' frames (ragged lengths) in ONE launch."""
    if not frames:
        return []
    I = interval_ms(interval)
    dev = _device()
    lens = [len(f) for f in frames]
    T = max(1, max(lens))
    S = len(frames)
    fields = [c for c in RESAMPLE_AGG if all(c in f.columns for f in frames)]
    ts = np.zeros((S, T), dtype=np.int64)
    host = {c: np.full((S, T), np.nan) for c in fields}
    for s, df in enumerate(frames):
        n = lens[s]
        if n == 0:
            continue
        t = pd.to_numeric(df["open_time"], errors="coerce").to_numpy(np.int64)
        if (np.diff(t) < 0).any():
            raise ValueError("resample: open_time must be ascending (pre_process sorts it)")
        ts[s, :n] = t
        ts[s, n:] = t[-1]
        for c in fields:
            host[c][s, :n] = pd.to_numeric(df[c], errors="coerce").to_numpy(np.float64)
    out_ts, outs, out_n = engine.resample(
        torch.from_numpy(ts).to(dev),
        {c: torch.from_numpy(host[c]).to(dev) for c in fields},
        {c: RESAMPLE_AGG[c] for c in fields},
        I,
        lens=torch.tensor(lens, dtype=torch.int64),
    )
    out_ts = out_ts.cpu().numpy()
    outs = {c: v.cpu().numpy() for c, v in outs.items()}
    out_n = out_n.cpu().numpy()
    res = []
    for s in range(S):
        n = int(out_n[s])
        d = {"open_time": out_ts[s, :n]}
        for c in fields:
            d[c] = outs[c][s, :n]
        r = pd.DataFrame(d)
        r.index = pd.to_datetime(r["open_time"], unit="ms")
        r.index.name = None
        res.append(r)
    return res
