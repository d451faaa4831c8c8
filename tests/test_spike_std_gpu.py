"""bq_spike_base_std's five rolling std columns (FailedSpikeFade
compute_base_features / compute_early_features, strategies/failed_spike_fade.py:
293-339: close and volume over the base window, close over 8 and 20, body size
pct over 10) against pandas' rolling().std() directly, on a panel with halted
stretches (constant prices, zero volume), spikes, missing closes and a
high-priced row — tests/spike_std.py's rule: 1e-9 of pandas, or closer to the
exact window std where pandas' online variance drifted — and the pass's other
columns equal to bq_spike_base's fed with the replayed stds wherever the
stds are equal."""

import numpy as np
import pandas as pd
import pytest
import torch

from binquant_amd import engine
from binquant_amd.synth import numpy_panel
from tests import spike_std

pytestmark = pytest.mark.gpu


def _panel():
    S, T = 24, 2300
    p = numpy_panel(S, T, seed0=202, edges=True)
    for s, (a, b) in enumerate(((300, 360), (1020, 1100), (2040, 2090))):
        for f in ("open", "high", "low", "close"):
            p[f][s, a:b] = p["close"][s, a]
        p["volume"][s, a:b] = 0.0
    p["close"][4, 700:703] = np.nan
    p["close"][5] = 3.1e4 * np.exp(np.cumsum(np.random.default_rng(1).normal(0, 1e-4, T)))   # high price, low vol
    p["open"][5] = np.r_[p["close"][5, 0], p["close"][5, :-1]]
    p["high"][5] = np.fmax(p["open"][5], p["close"][5]) * 1.00001
    p["low"][5] = np.fmin(p["open"][5], p["close"][5]) * 0.99999
    rng = np.random.default_rng(9)
    sp = rng.random((S, T)) < 0.01
    p["volume"][sp] *= 8.0
    return p


@pytest.mark.parametrize("W", [12, 3, 30])
def test_spike_std_columns_against_pandas(cuda, W):
    p = _panel()
    d = {k: torch.from_numpy(v).cuda() for k, v in p.items()}
    qv = d["volume"] * d["close"]
    (cf,) = engine.rolling_many(engine.Ffill(d["close"]))
    got = engine.spike_base_std(d["open"], d["high"], d["low"], d["close"], d["volume"], qv, cf, W, 3)
    g = {k: v.cpu().numpy() for k, v in got.items()}
    bsp = np.abs(p["close"] - p["open"]) / (p["open"] + 1e-6)
    np.testing.assert_array_equal(g["body_size_pct"], bsp)
    want = {}
    for col, (key, w) in spike_std.STD_COLS.items():
        x = {"close": p["close"], "volume": p["volume"], "body_size_pct": bsp}[key]
        w = W if w is None else w
        want[col] = np.stack([pd.Series(r).rolling(w).std().to_numpy() for r in x])
    # row 5 (price 3.1e4, 1e-4 moves): pandas' online variance drifts on most of
    # its short windows — every such position is checked against the exact std
    spike_std.check(g, want, {"close": p["close"], "volume": p["volume"], "body_size_pct": bsp}, base_window=W,
                    max_frac=0.1)
    # the rest of the pass equals bq_spike_base fed with these very std columns
    ref = engine.spike_base(d["open"], d["high"], d["low"], d["close"], d["volume"], qv, cf,
                            *(got[k] for k in engine.SPIKE_STD), W, 3)
    for k, v in ref.items():
        np.testing.assert_array_equal(v.cpu().numpy(), g[k], err_msg=k)
