"""GPU parity: bq_supertrend (Indicators.set_supertrend, strategies/coinrule/
coinrule.py:143-160) vs the oracle's band recursion (oracle/indicators_ref.py:
supertrend; pybinbot absent -> parity unpinned against pybinbot itself).

engine.supertrend forms the ATR in the kernel's own walk as a replay of
pandas' roll_mean (bq_supertrend_hlc), so flags and bands must equal the
oracle's bit for bit over every candle. With an ATR column from elsewhere
(bq_supertrend, here the enrich kernel's windowed ATR) the trend flag is a
state machine over comparisons, so it is compared exactly up to the first
candle whose decision lies within the 1e-9 tolerance band of its threshold (a
near-tie may legitimately flip and then propagate); the bands are compared
with the fp64 tolerance of tests/util.py over the same span.

Panel mode (engine.supertrend(exact=False), bq_supertrend_panel): lanes walk
chunks of a row from a warm-up and a serial pass re-walks every chunk whose
guessed start state differs from its predecessor's end state, so its flags and
bands must equal the sequential recursion on the panel kernel's own ATR (a
direct window sum in time order) bit for bit — checked against that
restatement (panel_ref below) on panels where ~0.4 % of the warm-ups end in a
wrong state (the re-walk runs) — and the oracle's within the tie rule above.
"""

import numpy as np
import pandas as pd
import pytest
import torch

from binquant_amd import engine
from binquant_amd.indicators import Indicators
from binquant_amd.synth import numpy_panel
from oracle import indicators_ref as ref
from tests.util import assert_close

pytestmark = pytest.mark.gpu


def oracle_panel(panel, period, mult):
    S, T = panel["close"].shape
    out = {k: np.empty((S, T)) for k in ("supertrend", "supertrend_upper", "supertrend_lower")}
    out["supertrend"] = np.empty((S, T), dtype=bool)
    tie_free = np.full(S, T)
    for s in range(S):
        df = pd.DataFrame({k: panel[k][s] for k in ("open", "high", "low", "close", "volume")})
        df = ref.supertrend(df, mult, period)
        for k in out:
            out[k][s] = df[k].to_numpy()
        c = panel["close"][s]
        up_p, lo_p = out["supertrend_upper"][s][:-1], out["supertrend_lower"][s][:-1]
        tol = 1e-9 * np.abs(c[1:])
        near = (np.abs(c[1:] - up_p) <= tol) | (np.abs(c[1:] - lo_p) <= tol)
        if near.any():
            tie_free[s] = int(np.argmax(near)) + 1
    return out, tie_free


def run(panel, period=10, mult=3.0, atr_input=False, exact=True):
    t = {k: torch.from_numpy(np.ascontiguousarray(v)).cuda() for k, v in panel.items()}
    atr = None
    if atr_input:
        zero = torch.zeros_like(t["close"])
        atr = engine.enrich(t["close"], t["high"], t["low"], t["close"], zero,
                            params=engine.IndicatorParams(atr_window=period), columns=("ATR",))["ATR"]
    r = engine.supertrend(t["high"], t["low"], t["close"], period=period, multiplier=mult, atr=atr, exact=exact)
    torch.cuda.synchronize()
    return {k: v.cpu().numpy() for k, v in r.items()}


CASES = [(70, 700, 10, 3.0), (3, 1, 10, 3.0), (5, 9, 10, 3.0), (64, 257, 7, 2.0), (130, 33, 14, 1.5),
         (1, 2000, 10, 3.0), (65, 300, 1, 3.0), (9, 500, 16, 3.0), (9, 500, 126, 2.5)]


@pytest.mark.parametrize("S,T,period,mult", CASES)
@pytest.mark.parametrize("edges", [False, True])
def test_supertrend_bit_exact(cuda, S, T, period, mult, edges):
    """Fused ATR: every flag and band equals the oracle's (NaN candles, halts
    and gaps included with edges=True)."""
    panel = numpy_panel(S, T, seed0=S + T + period, edges=edges)
    got = run(panel, period, mult)
    want, _ = oracle_panel(panel, period, mult)
    for k in want:
        np.testing.assert_array_equal(got[k], want[k], err_msg=k)


@pytest.mark.parametrize("S,T,period,mult", CASES[:6])
def test_supertrend_atr_input_matches_oracle(cuda, S, T, period, mult):
    panel = numpy_panel(S, T, seed0=S + T + period, edges=False)
    got = run(panel, period, mult, atr_input=True)
    want, n_ok = oracle_panel(panel, period, mult)
    price = np.abs(panel["close"]).mean(axis=1, keepdims=True)
    for s in range(S):
        n = n_ok[s]
        np.testing.assert_array_equal(got["supertrend"][s, :n], want["supertrend"][s, :n], err_msg=f"symbol {s}")
        for k in ("supertrend_upper", "supertrend_lower"):
            assert_close(got[k][s, :n], want[k][s, :n], f"{k}[{s}]", scale=price[s])
    assert (n_ok == T).mean() > 0.9   # near-ties are rare on random walks


def test_supertrend_flips_on_trend_and_holds_bands(cuda):
    """Rally then sell-off: the flag must be up at the top and down at the end,
    and the held lower band must never fall while the trend stays up."""
    T = 300
    close = np.concatenate([np.linspace(100, 160, 150), np.linspace(160, 90, 150)])
    panel = {"open": np.r_[close[0], close[:-1]][None], "close": close[None],
             "high": (close * 1.002)[None], "low": (close * 0.998)[None], "volume": np.ones((1, T))}
    got = run(panel)
    want, _ = oracle_panel(panel, 10, 3.0)
    np.testing.assert_array_equal(got["supertrend"], want["supertrend"])
    assert got["supertrend"][0, 149] and not got["supertrend"][0, -1]
    lo = got["supertrend_lower"][0, 10:150]
    assert (np.diff(lo) >= 0).all()


def test_supertrend_constant_market_is_exact(cuda):
    """A halted market (h == l == c) has ATR exactly 0 in both paths, so the
    bands equal the price and every comparison is an exact tie resolved the
    same way (hold)."""
    T = 80
    c = np.full(T, 0.3)
    c[:20] = np.linspace(0.29, 0.31, 20)
    panel = {"open": c[None], "high": c[None].copy(), "low": c[None].copy(), "close": c[None], "volume": np.ones((1, T))}
    got = run(panel)
    want, _ = oracle_panel(panel, 10, 3.0)
    np.testing.assert_array_equal(got["supertrend"], want["supertrend"])
    np.testing.assert_array_equal(got["supertrend_upper"][0, 40:], want["supertrend_upper"][0, 40:])


def test_set_supertrend_dataframe_api(cuda):
    panel = numpy_panel(1, 400, seed0=5, edges=False)
    df = pd.DataFrame({k: v[0] for k, v in panel.items()})
    out = Indicators.set_supertrend(df, multiplier=3.0)
    assert out is df and out["supertrend"].dtype == bool
    want = ref.supertrend(pd.DataFrame({k: v[0] for k, v in panel.items()}), 3.0, 10)
    assert bool(out["supertrend"].iloc[-1]) == bool(want["supertrend"].iloc[-1])


def panel_ref(h, l, c, period, mult):
    """The panel kernel's arithmetic, restated: TR (skip-NaN max), ATR = the
    window's TR summed in time order / period (min_periods = period, an
    all-equal window gives the value), raw bands hl2 +- mult * ATR, then the
    band recursion of oracle.indicators_ref.supertrend."""
    T = len(c)
    pc = np.r_[np.nan, c[:-1]]
    tr = np.fmax(h - l, np.fmax(np.abs(h - pc), np.abs(l - pc)))
    atr = np.full(T, np.nan)
    for t in range(period - 1, T):
        w = tr[t - period + 1 : t + 1]
        s, n = 0.0, 0
        for v in w:
            if v == v:
                s += v
                n += 1
        if n < period:
            continue
        atr[t] = w[0] if np.all(w == w[0]) else s / period
    hl2 = (h + l) / 2.0
    m = mult * atr
    upper, lower = hl2 + m, hl2 - m
    up = np.ones(T, dtype=bool)
    for t in range(1, T):
        p = t - 1
        if c[t] > upper[p]:
            up[t] = True
        elif c[t] < lower[p]:
            up[t] = False
        else:
            up[t] = up[p]
            if up[t] and lower[t] < lower[p]:
                lower[t] = lower[p]
            if not up[t] and upper[t] > upper[p]:
                upper[t] = upper[p]
    return up, upper, lower


@pytest.mark.parametrize("S,T,period,mult,edges", [(64, 2000, 10, 3.0, False), (24, 2048, 10, 3.0, True),
                                                   (40, 700, 7, 2.0, True), (5, 9, 10, 3.0, False),
                                                   (70, 130, 14, 1.5, False), (3, 1, 10, 3.0, False),
                                                   (9, 500, 126, 2.5, False), (2, 5000, 10, 3.0, True),
                                                   (256, 2000, 10, 3.0, False), (4, 1500, 14, 3.0, True)])
def test_supertrend_panel_equals_recursion_on_its_atr(cuda, S, T, period, mult, edges):
    """Panel mode bit for bit against the sequential recursion on the same ATR
    (panel_ref); rows longer than 2048 candles run the exact kernel (oracle)."""
    panel = numpy_panel(S, T, seed0=S * 7 + T + period, edges=edges)
    got = run(panel, period, mult, exact=False)
    for s in range(S):
        if T > 2048:
            want, _ = oracle_panel({k: v[s:s + 1] for k, v in panel.items()}, period, mult)
            want = (want["supertrend"][0], want["supertrend_upper"][0], want["supertrend_lower"][0])
        else:
            want = panel_ref(panel["high"][s], panel["low"][s], panel["close"][s], period, mult)
        for k, w in zip(("supertrend", "supertrend_upper", "supertrend_lower"), want):
            np.testing.assert_array_equal(got[k][s], w, err_msg=f"{k}[{s}]")


def test_supertrend_panel_matches_oracle(cuda):
    """Panel mode against the oracle (pandas' Kahan ATR): flags equal up to the
    first near-tie, bands within the fp64 tolerance."""
    S, T = 64, 2000
    panel = numpy_panel(S, T, seed0=1234, edges=False)   # (halted stretches are exact ties: panel_ref covers them)
    got = run(panel, 10, 3.0, exact=False)
    want, n_ok = oracle_panel(panel, 10, 3.0)
    price = np.abs(np.nan_to_num(panel["close"])).max(axis=1, keepdims=True)
    for s in range(S):
        n = n_ok[s]
        np.testing.assert_array_equal(got["supertrend"][s, :n], want["supertrend"][s, :n], err_msg=f"symbol {s}")
        for k in ("supertrend_upper", "supertrend_lower"):
            assert_close(got[k][s, :n], want[k][s, :n], f"{k}[{s}]", scale=price[s])
    assert (n_ok == T).mean() > 0.9
