"""The pybinbot.Indicators-compatible DataFrame surface (binquant_amd.indicators)
vs the oracle restatement; CPU tests cover argument validation only."""

import numpy as np
import pandas as pd
import pytest

from binquant_amd.indicators import Indicators, enrich_frames, indicators_enrichment
from binquant_amd.synth import numpy_symbol
from oracle import indicators_ref as ref
from tests.util import assert_close


def frame(T=400, seed=0, scale=100.0):
    return pd.DataFrame(numpy_symbol(T, seed, scale=scale))


def test_missing_close_raises_value_error():
    df = frame().drop(columns=["close"])
    with pytest.raises(ValueError, match="close"):
        Indicators.rsi(df)


def test_missing_high_raises_value_error():
    df = frame().drop(columns=["high"])
    with pytest.raises(ValueError, match="high"):
        Indicators.atr(df, window=14)


def test_window_out_of_range():
    with pytest.raises(ValueError):
        Indicators.moving_averages(frame(), 500)


@pytest.mark.gpu
def test_each_indicator_matches_oracle(cuda):
    base = frame(600, 3)
    price = float(base["close"].abs().mean())
    cases = [
        (lambda d: Indicators.moving_averages(d, 7), lambda d: ref.moving_averages(d, 7), ["ma_7"]),
        (lambda d: Indicators.moving_averages(d, 100), lambda d: ref.moving_averages(d, 100), ["ma_100"]),
        (lambda d: Indicators.macd(df=d), lambda d: ref.macd(d), ["macd", "macd_signal"]),
        (lambda d: Indicators.rsi(df=d), lambda d: ref.rsi(d), ["rsi"]),
        (lambda d: Indicators.bollinguer_spreads(d), lambda d: ref.bollinguer_spreads(d), ["bb_upper", "bb_mid", "bb_lower"]),
        (lambda d: Indicators.set_twap(d), lambda d: ref.set_twap(d), ["twap"]),
        (lambda d: Indicators.atr(df=d, window=14), lambda d: ref.atr(d, 14), ["ATR"]),
    ]
    for ours, theirs, cols in cases:
        g = ours(base.copy())
        w = theirs(base.copy())
        for c in cols:
            assert_close(g[c].to_numpy(), w[c].to_numpy(), c, scale=100.0 if c == "rsi" else price)
    assert Indicators.mfi(base.copy()) == pytest.approx(ref.mfi(base.copy()), rel=1e-9, abs=1e-9)


@pytest.mark.gpu
def test_enrichment_composition_and_ragged_batch(cuda):
    frames = [frame(n, seed=n) for n in (150, 400, 999, 1)]
    want = [ref.indicators_enrichment(f.copy()) for f in frames]
    got = enrich_frames([f.copy() for f in frames])
    for g, w in zip(got, want):
        price = float(w["close"].abs().mean())
        for c in ref.CANONICAL:
            assert_close(g[c].to_numpy(), w[c].to_numpy(), c, scale=100.0 if c in ("rsi", "mfi") else price)
    one = indicators_enrichment(frames[1].copy())
    w = ref.ma_spreads(ref.indicators_enrichment(frames[1].copy()))
    for c in ("big_ma_spread", "small_ma_spread"):
        assert_close(one[c].to_numpy(), w[c].to_numpy(), c, scale=1.0)


def _pin_frame(case):
    """The reference's own make_ohlcv_df(n=50, oversold=...) frame
    (tests/test_coinrule_price_tracker.py:148-189; tests/golden/ohlcv_pins.npz)."""
    from pathlib import Path

    z = np.load(Path(__file__).resolve().parent / "golden" / "ohlcv_pins.npz")
    return pd.DataFrame({k: z[f"{case}__{k}"] for k in ("open", "high", "low", "close", "volume", "close_time")})


@pytest.mark.gpu
@pytest.mark.parametrize("case", ["oversold", "uptrend"])
def test_reference_make_ohlcv_df_pins(cuda, case):
    """The reference's Indicators.mfi pins (test_coinrule_price_tracker.py:226-248:
    a float in [0, 100], < 50 on the oversold frame) and make_ohlcv_df's
    docstring (the oversold frame gives RSI < 30 and a negative MACD; the
    uptrend "will not be below 30"), through the GPU drop-in on the
    reference's own frames, and equal to the oracle restatement."""
    df = _pin_frame(case)
    m = Indicators.mfi(df.copy())
    assert isinstance(m, float) and 0.0 <= m <= 100.0
    assert m == pytest.approx(ref.mfi(df.copy()), rel=1e-9, abs=1e-9)
    rsi = Indicators.rsi(df=df.copy())["rsi"].iloc[-1]
    macd = Indicators.macd(df=df.copy())["macd"].iloc[-1]
    assert rsi == pytest.approx(ref.rsi(df.copy())["rsi"].iloc[-1], rel=1e-9, abs=1e-9)
    assert macd == pytest.approx(ref.macd(df.copy())["macd"].iloc[-1], rel=1e-9, abs=1e-12)
    if case == "oversold":
        assert m < 50.0 and rsi < 30.0 and macd < 0.0
    else:
        assert rsi >= 30.0 and macd > 0.0
    full = indicators_enrichment(df.copy())
    want = ref.indicators_enrichment(df.copy())
    for c in ref.CANONICAL:
        assert_close(full[c].to_numpy(), want[c].to_numpy(), c, scale=100.0)


def test_oracle_on_reference_make_ohlcv_df_pins():
    """The oracle restatement itself satisfies the reference's pins on the
    reference's frames (CPU): MFI float in [0, 100], < 50 oversold; RSI < 30
    and MACD < 0 oversold."""
    for case in ("oversold", "uptrend"):
        df = _pin_frame(case)
        m = ref.mfi(df.copy())
        assert isinstance(m, float) and 0.0 <= m <= 100.0
        e = ref.indicators_enrichment(df.copy())
        if case == "oversold":
            assert m < 50.0 and e["rsi"].iloc[-1] < 30.0 and e["macd"].iloc[-1] < 0.0
        else:
            assert e["rsi"].iloc[-1] >= 30.0 and e["macd"].iloc[-1] > 0.0


@pytest.mark.gpu
def test_mfi_bounds_like_reference_test(cuda):
    """tests/test_coinrule_price_tracker.py:226-248: MFI in [0, 100] and < 50
    on a low-volume downtrend."""
    n = 60
    close = np.linspace(100, 80, n)
    df = pd.DataFrame({"open": close + 0.2, "high": close + 0.5, "low": close - 0.5, "close": close,
                       "volume": np.linspace(1000, 100, n)})
    v = Indicators.mfi(df)
    assert 0.0 <= v <= 100.0 and v < 50.0
