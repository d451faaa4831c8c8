"""pandas' window operations treat +-inf as missing: rolling(...) and
ewm(...) run on np.where(np.isinf(values), np.nan, values)
(BaseWindow._prep_values, pandas/core/window/rolling.py). Strategy series
that feed windows are ratios (relative volume v / mean over a zero-volume
stretch, pct changes after a zero close) and do reach +-inf, so every rolling
kernel family reads its inputs through that rule (bq_device.h win_val):
the exact replays (mean / sum / var / std / ewm: bit for bit with pandas),
panel mode (sums / means / ewm within rounding), the order-statistic kernels
(lane, stencil, tile, sorted-register slide), while ffill keeps infinities
as pandas does."""

import numpy as np
import pandas as pd
import pytest
import torch

pytestmark = pytest.mark.gpu


def _series(S, T, seed):
    rng = np.random.default_rng(seed)
    x = 100.0 + np.cumsum(rng.normal(0, 1, (S, T)), axis=1)
    for r in range(S):
        idx = rng.choice(T, size=max(2, T // 50), replace=False)
        x[r, idx[: len(idx) // 2]] = np.inf
        x[r, idx[len(idx) // 2:]] = -np.inf
    x[0, 5:40] = np.nan
    x[1, : T // 3] = np.inf   # a long stretch of infinities
    return x


def _pandas(x, spec):
    s = pd.Series(x)
    kind = spec[0]
    if kind == "ewm":
        _, kw = spec
        return s.ewm(adjust=False, **kw).mean().to_numpy()
    if kind == "ffill":
        return s.ffill().to_numpy()
    _, w, stat, kw = spec
    return getattr(s.rolling(w, **kw), stat)().to_numpy()


SPECS = [("roll", 5, "mean", {}), ("roll", 12, "std", {}), ("roll", 20, "sum", {"min_periods": 1}),
         ("roll", 10, "var", {"min_periods": 3}), ("roll", 19, "median", {}), ("roll", 48, "max", {}),
         ("roll", 6, "min", {}), ("ewm", {"span": 20}), ("ewm", {"alpha": 1 / 14, "min_periods": 14}),
         ("ffill",)]


def _device(engine, d, spec, exact):
    E, R, FF = engine.Ewm, engine.Roll, engine.Ffill
    if spec[0] == "ewm":
        return engine.rolling_many(E(d, **spec[1]), exact=exact)[0]
    if spec[0] == "ffill":
        return engine.rolling_many(FF(d), exact=exact)[0]
    _, w, stat, kw = spec
    return engine.rolling_many(R(d, w, stat, min_periods=kw.get("min_periods")), exact=exact)[0]


def _check(got, want, name, exact):
    np.testing.assert_array_equal(np.isnan(got), np.isnan(want), err_msg=name)
    m = ~np.isnan(want)
    inf = np.isinf(want)
    np.testing.assert_array_equal(got[inf], want[inf], err_msg=name)
    f = m & ~inf
    if exact:
        np.testing.assert_array_equal(got[f], want[f], err_msg=name)
    else:
        sc = max(1.0, float(np.max(np.abs(want[f])))) if f.any() else 1.0
        assert np.all(np.abs(got[f] - want[f]) <= 1e-9 * np.abs(want[f]) + 1e-12 * sc), name


@pytest.mark.parametrize("exact", [True, False])
def test_window_ops_skip_infinities(cuda, exact):
    from binquant_amd import engine

    S, T = 6, 700
    x = _series(S, T, 3)
    d = torch.from_numpy(x).cuda()
    for spec in SPECS:
        got = _device(engine, d, spec, exact).cpu().numpy()
        for r in range(S):
            # exact mode equals pandas bit for bit (replays, order statistics); panel
            # mode's sums / means / ewm agree to rounding
            _check(got[r], _pandas(x[r], spec), f"{spec} row {r} exact={exact}", exact or spec[0] == "ffill")


@pytest.mark.parametrize("w,q", [(48, 0.8), (60, 0.85), (80, 0.92), (19, 0.5)])
def test_quantile_kernels_skip_infinities(cuda, w, q):
    """Large panel (the sorted-register slide kernel) and a small one (tile /
    stencil kernels): rolling quantiles with +-inf in the windows."""
    from binquant_amd import engine

    for S, T in ((2200, 2000), (5, 600)):
        x = _series(S, T, w)
        d = torch.from_numpy(x).cuda()
        for exact in (True, False):
            got = engine.rolling_many(engine.Roll(d, w, "quantile", q=q, min_periods=w // 3), exact=exact)[0]
            got = got.cpu().numpy()
            for r in range(0, S, max(1, S // 12)):
                want = pd.Series(x[r]).rolling(w, min_periods=w // 3).quantile(q).to_numpy()
                _check(got[r], want, f"q{q} w{w} S{S} row {r} exact={exact}", False)
