"""pandas restatement of the frame plumbing around the indicator path
(SURVEY §8a a9, §8f row 4). TEST INFRASTRUCTURE ONLY (see oracle/__init__.py).

* resample: pybinbot Candles.resample(df, interval="1h")
  (producers/context_evaluator.py:403-407; pybinbot absent -> the standard
  OHLCV aggregation of pandas' resample on the open_time DatetimeIndex,
  parity unpinned against pybinbot).
* left_merge: strategies/liquidation_sweep_pump.py:255-263 (verbatim pandas
  calls: drop_duplicates("open_time", keep="last"), merge how="left").
* joined_returns / beta_corr_last: producers/context_evaluator.py:161-194
  (log returns per frame, inner join on the index, dropna, rolling cov/var/corr).
"""

from __future__ import annotations

import numpy as np
import pandas as pd


def resample(df: pd.DataFrame, interval: str, agg: dict[str, str]) -> pd.DataFrame:
    d = df.copy()
    d.index = pd.to_datetime(d["open_time"].astype("int64"), unit="ms")
    cols = {c: a for c, a in agg.items() if c in d.columns}
    r = d[list(cols)].resample(interval).agg(cols)
    r.insert(0, "open_time", r.index.astype("int64") // 10**6)
    return r


def left_merge(open_time: np.ndarray, bench_open_time: np.ndarray, bench_close: np.ndarray) -> np.ndarray:
    result = pd.DataFrame({"open_time": np.asarray(open_time, dtype=np.int64)})
    btc_by_open_time = pd.DataFrame(
        {"open_time": np.asarray(bench_open_time).astype("int64"), "btc_close": np.asarray(bench_close, float)}
    ).drop_duplicates("open_time", keep="last")
    return result[["open_time"]].merge(btc_by_open_time, on="open_time", how="left", sort=False)[
        "btc_close"
    ].to_numpy()


def joined_returns(ts, close, bench_ts, bench_close) -> pd.DataFrame:
    """Frames indexed by open_time; returns on each frame's own rows."""
    alt = pd.DataFrame({"close": np.asarray(close, float)}, index=np.asarray(ts, np.int64))
    btc = pd.DataFrame({"close": np.asarray(bench_close, float)}, index=np.asarray(bench_ts, np.int64))
    btc["returns"] = np.log(btc["close"] / btc["close"].shift(1))
    alt["returns"] = np.log(alt["close"] / alt["close"].shift(1))
    returns = alt[["returns"]].join(btc["returns"], how="inner", rsuffix="_btc").dropna()
    returns.columns = ["alt", "btc"]
    return returns


def beta_corr_series(returns: pd.DataFrame, window: int = 50) -> tuple[np.ndarray, np.ndarray]:
    cov = returns["alt"].rolling(window).cov(returns["btc"])
    var = returns["btc"].rolling(window).var()
    beta = cov / var.replace(0, np.nan)
    corr = returns["alt"].rolling(window).corr(returns["btc"])
    return beta.to_numpy(), corr.to_numpy()
