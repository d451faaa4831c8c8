"""CPU checks of the Candles drop-in: the behaviour the
reference's own tests/test_ohlc.py pins for pybinbot.Candles.ensure_ohlc
(same frame, same expectations), plus pre_process / post_process / interval
parsing of the restatement (no device needed)."""

import numpy as np
import pandas as pd
import pytest
from pandas.api.types import is_numeric_dtype

from binquant_amd.candles import Candles, interval_ms


def base_df():
    # the frame of tests/test_ohlc.py:7-22
    return pd.DataFrame(
        {
            "open": [1.0, 2.0, 3.0],
            "high": [1.5, 2.5, 3.5],
            "low": [0.5, 1.5, 2.5],
            "close": [1.2, 2.2, 3.2],
            "open_time": [1000, 2000, 3000],
            "close_time": [1500, 2500, 3500],
            "volume": [10, 20, 30],
            "quote_asset_volume": [100, 200, 300],
            "number_of_trades": [1, 2, 3],
            "taker_buy_base_asset_volume": [5, 10, 15],
            "taker_buy_quote_asset_volume": [50, 100, 150],
        }
    )


def helper():
    return Candles(exchange="binance", candles=[])


def test_ensure_ohlc_success():
    assert isinstance(helper().ensure_ohlc(base_df()), pd.DataFrame)


def test_ensure_ohlc_missing_columns_named():
    with pytest.raises(ValueError) as exc:
        helper().ensure_ohlc(base_df().drop(columns=["volume", "close_time"]))
    assert "volume" in str(exc.value) and "close_time" in str(exc.value)


def test_ensure_ohlc_coerces_strings():
    df = base_df().astype({c: "string" for c in ("open", "high", "low", "close")})
    v = helper().ensure_ohlc(df)
    for c in ("open", "high", "low", "close"):
        assert is_numeric_dtype(v[c])


def test_quote_asset_volume_all_nan_rejected():
    df = base_df()
    df["quote_asset_volume"] = ["x", "y", "z"]
    with pytest.raises(ValueError) as exc:
        helper().ensure_ohlc(df)
    assert "quote_asset_volume" in str(exc.value)


def binance_rows(n=6, start=1_700_000_000_000, step=900_000):
    rows = []
    for i in range(n):
        t = start + i * step
        p = 100 + i
        rows.append([t, str(p), str(p + 1), str(p - 1), str(p + 0.5), "12.5", t + step - 1, "1250.0", 7, "6.0", "600.0", "0"])
    return rows


def test_pre_process_rows_sorted_deduplicated_numeric():
    rows = binance_rows()
    dup = list(rows[2])
    dup[4] = "999.0"                      # a later update of the same candle wins
    rows = [rows[3], rows[0], rows[2], rows[1], dup, rows[5], rows[4]]
    df = Candles(exchange="binance", candles=rows).pre_process()
    assert list(df["open_time"]) == sorted(set(r[0] for r in rows))
    assert df["close"].dtype == np.float64 and df["open_time"].dtype == np.int64
    assert df.loc[2, "close"] == 999.0
    assert list(df.index) == list(range(len(df)))


def test_pre_process_kucoin_layout():
    rows = [[1_700_000_000 + 900 * i, "1", "2", "3", "0.5", "10", "20"] for i in range(3)]
    df = Candles(exchange="kucoin", candles=rows).pre_process()
    assert df.loc[0, "open_time"] == 1_700_000_000_000
    assert (df["close"] == 2.0).all() and (df["high"] == 3.0).all()


def test_pre_process_empty():
    assert Candles(exchange="binance", candles=[]).pre_process().empty


def test_post_process_drops_warmup_rows():
    df = base_df()
    df["ma_2"] = df["close"].rolling(2).mean()
    out = helper().post_process(df)
    assert len(out) == 2 and list(out.index) == [0, 1]


@pytest.mark.parametrize("s,ms", [("1h", 3_600_000), ("15m", 900_000), ("4h", 14_400_000), ("1d", 86_400_000),
                                  ("15min", 900_000), (60_000, 60_000)])
def test_interval_parsing(s, ms):
    assert interval_ms(s) == ms


def test_interval_rejects_unknown():
    with pytest.raises(ValueError):
        interval_ms("3 fortnights")
