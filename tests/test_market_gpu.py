"""GPU parity of the market-context path: bq_market_features (per-symbol
features of _compute_symbol_features at every timestamp under the
MarketStateStore history cap) and bq_breadth_partial (the _build_context sums)."""

import numpy as np
import pytest
import torch

from binquant_amd import engine
from binquant_amd._lib import FEATURE_COLUMNS
from binquant_amd.synth import numpy_panel
from oracle import market_ref
from tests.util import assert_close

pytestmark = pytest.mark.gpu


def gpu_feats(panel, max_bars):
    d = {k: torch.from_numpy(v).cuda() for k, v in panel.items()}
    f = engine.market_features(d["high"], d["low"], d["close"], max_bars=max_bars)
    torch.cuda.synchronize()
    return d, f


@pytest.mark.parametrize("S,T,M", [(6, 700, 400), (4, 1500, 200), (3, 2100, 512), (5, 60, 15)])
def test_features_match_reference_restatement(cuda, S, T, M):
    panel = numpy_panel(S, T, seed0=T + M)
    _, f = gpu_feats(panel, M)
    f = {k: v.cpu().numpy() for k, v in f.items()}
    rng = np.random.default_rng(0)
    ts = sorted(set([0, 1, 2, 13, 14, 19, 20, M - 1, M, M + 1, T - 1] + rng.integers(0, T, 40).tolist()))
    ts = [t for t in ts if 0 <= t < T]
    for s in range(S):
        for t in ts:
            want = market_ref.panel_features_at(panel["high"][s], panel["low"][s], panel["close"][s], t, M)
            if want is None:
                assert all(np.isnan(f[k][s, t]) for k in FEATURE_COLUMNS)
                continue
            got = {k: f[k][s, t] for k in FEATURE_COLUMNS}
            for k in FEATURE_COLUMNS:
                assert_close([got[k]], [want[k]], f"{k}[{s},{t}]", rtol=1e-9, scale=[1e-3])
            c = panel["close"][s, t]
            for e in ("ema20", "ema50"):
                if abs(c - want[e]) > 1e-9 * abs(c):
                    assert (c > got[e]) == want[f"above_{e}"]


def test_breadth_partial_is_the_symbol_sum(cuda):
    S, T = 200, 500
    panel = numpy_panel(S, T, seed0=1)
    d, f = gpu_feats(panel, 400)
    part = engine.breadth_partial(d["close"], f).cpu().numpy()
    fn = {k: v.cpu().numpy() for k, v in f.items()}
    c = panel["close"]
    valid = ~np.isnan(fn["return_pct"])
    np.testing.assert_array_equal(part[:, 0], valid.sum(axis=0))
    np.testing.assert_array_equal(part[:, 1], (valid & (fn["return_pct"] > 0)).sum(axis=0))
    np.testing.assert_array_equal(part[:, 2], (valid & (fn["return_pct"] < 0)).sum(axis=0))
    np.testing.assert_array_equal(part[:, 3], (valid & (c > fn["ema20"])).sum(axis=0))
    np.testing.assert_array_equal(part[:, 4], (valid & (c > fn["ema50"])).sum(axis=0))
    for i, k in ((5, "return_pct"), (6, "trend_score"), (7, "atr_pct"), (8, "bb_width")):
        want = np.where(valid, fn[k], 0.0).sum(axis=0)
        assert_close(part[:, i], want, k, rtol=1e-12, scale=np.abs(np.where(valid, fn[k], 0)).sum(axis=0) + 1e-300)
    # deterministic: a second run is bitwise identical
    part2 = engine.breadth_partial(d["close"], f).cpu().numpy()
    np.testing.assert_array_equal(part, part2)
