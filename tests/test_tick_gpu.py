"""GPU parity of the streaming tick path (bq_state_seed + bq_tick) against
the pandas oracle on the full series: tick t must equal row t of
indicators_enrichment over candles [0, t]."""

import numpy as np
import pytest
import torch

from binquant_amd import engine
from binquant_amd.synth import numpy_panel
from oracle import indicators_ref as ref
from tests.util import assert_close

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("S,T0,N", [(64, 400, 60), (8, 1, 130), (300, 150, 5)])
def test_tick_matches_full_series(cuda, S, T0, N):
    T = T0 + N
    panel = numpy_panel(S, T, seed0=S + T)
    want = ref.enrich_panel(panel["open"], panel["high"], panel["low"], panel["close"], panel["volume"])
    dev = {k: torch.from_numpy(v).cuda() for k, v in panel.items()}
    st = engine.TickState(S)
    st.seed(*(dev[k][:, :T0] for k in ("open", "high", "low", "close", "volume")))
    assert st.count == T0
    price = np.abs(panel["close"]).mean(axis=1)
    for t in range(T0, T):
        out = st.tick([dev[k][:, t].contiguous() for k in ("open", "high", "low", "close", "volume")])
        torch.cuda.synchronize()
        for k in ref.CANONICAL:
            scale = 100.0 if k in ("rsi", "mfi") else price
            assert_close(out[k].cpu().numpy(), want[k][:, t], f"{k}@{t}", scale=scale)
    assert st.count == T
    # EMAs are the exact pandas recursion once seeded: bitwise equal
    np.testing.assert_array_equal(out["ema20"].cpu().numpy(), want["ema20"][:, -1])


def _run_ticks(panel, T0, on_tick):
    dev = {k: torch.from_numpy(np.ascontiguousarray(v)).cuda() for k, v in panel.items()}
    S, T = panel["close"].shape
    st = engine.TickState(S)
    st.seed(*(dev[k][:, :T0] for k in ("open", "high", "low", "close", "volume")))
    for t in range(T0, T):
        out = st.tick([dev[k][:, t].contiguous() for k in ("open", "high", "low", "close", "volume")])
        torch.cuda.synchronize()
        on_tick(t, {k: v.cpu().numpy() for k, v in out.items()})
    assert st.count == T


def test_c3_ten_thousand_symbols(cuda):
    """BASELINE configs[2] (C3): 10 000 symbols seeded with 400 bars (the
    MarketStateStore cap, klines_provider.py:40), 24 ticks of one candle per
    symbol. Every column at 96 symbols spread over the panel (incl. the first
    and last) against the per-frame pandas oracle; the EMA family (ema20,
    ema50, macd, macd_signal) bit-exact on all 10 000 symbols at every tick."""
    S, T0, N = 10_000, 400, 24
    T = T0 + N
    panel = numpy_panel(S, T, seed0=3)
    sample = np.unique(np.r_[0, S - 1, np.linspace(0, S - 1, 94).astype(int)])
    want = ref.enrich_panel(*(panel[k][sample] for k in ("open", "high", "low", "close", "volume")))
    ema = ref.ema_family_panel(panel["close"])
    price = np.abs(panel["close"][sample]).mean(axis=1)
    seen = []

    def check(t, out):
        for k in ref.CANONICAL:
            scale = 100.0 if k in ("rsi", "mfi") else price
            assert_close(out[k][sample], want[k][:, t], f"{k}@{t}", scale=scale)
        for k in ("ema20", "ema50", "macd", "macd_signal"):
            np.testing.assert_array_equal(out[k], ema[k][:, t], err_msg=f"{k}@{t}")
        seen.append(t)

    _run_ticks(panel, T0, check)
    assert len(seen) == N


def test_tick_nan_candles_follow_pandas(cuda):
    """A symbol without a candle in a tick (NaN in all five fields) gives what
    pandas gives for that NaN row: EMAs hold and decay their old weight
    (ewm(adjust=False, ignore_na=False)), windows containing it are NaN, RSI /
    MFI count it as no move. Also NaN rows inside the seed history."""
    S, T0, N = 48, 160, 140
    T = T0 + N
    panel = numpy_panel(S, T, seed0=91)
    g = np.random.default_rng(4)
    for s in range(0, S, 3):
        for t in g.choice(np.arange(1, T), size=4, replace=False):
            for k in panel:
                panel[k][s, t] = np.nan
    for k in panel:   # a two-candle gap in the live ticks and one at the seed end
        panel[k][1, T0 + 30 : T0 + 32] = np.nan
        panel[k][2, T0 - 1] = np.nan
    want = ref.enrich_panel(*(panel[k] for k in ("open", "high", "low", "close", "volume")))
    price = np.nanmean(np.abs(panel["close"]), axis=1)

    def check(t, out):
        for k in ref.CANONICAL:
            scale = 100.0 if k in ("rsi", "mfi") else price
            assert_close(out[k], want[k][:, t], f"{k}@{t}", scale=scale)
        for k in ("ema20", "ema50", "macd", "macd_signal"):
            np.testing.assert_array_equal(out[k], want[k][:, t], err_msg=f"{k}@{t}")

    _run_ticks(panel, T0, check)
