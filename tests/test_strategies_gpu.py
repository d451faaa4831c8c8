"""a17/a18: strategy feature pipelines (bq_rolling / bq_ewm kernels + device
glue) vs the reference's own outputs (tests/golden/activity_burst.npz,
liquidation_sweep.npz from strategies/activity_burst_pump.py:51-158 and
strategies/liquidation_sweep_pump.py:195-269), and the rolling primitives vs
pandas on larger panels."""

from pathlib import Path

import numpy as np
import pandas as pd
import pytest
import torch

from tests.util import assert_close

G = Path(__file__).resolve().parent / "golden"
pytestmark = pytest.mark.gpu


def _cmp(got, want, name):
    if got.dtype == torch.bool:
        np.testing.assert_array_equal(got.cpu().numpy().astype(float).ravel(), want, err_msg=name)
    else:
        g = got.cpu().numpy().ravel()
        scale = np.nanmax(np.abs(want)) if np.isfinite(want).any() else 1.0
        assert_close(g, want, name, rtol=1e-9, scale=scale)


@pytest.mark.parametrize("case", ["with_quote", "no_quote"])
def test_activity_burst_matches_reference(cuda, case):
    from binquant_amd.strategies import activity_burst_features

    z = np.load(G / "activity_burst.npz")
    col = lambda k: torch.from_numpy(z[f"{case}__{k}"])[None].cuda()  # noqa: E731
    qv = col("quote_asset_volume") if f"{case}__quote_asset_volume" in z.files else None
    out = activity_burst_features(col("open"), col("high"), col("low"), col("close"), col("volume"), qv)
    for k, v in out.items():
        want = z[f"{case}__{k}"]
        _cmp(v if v.dim() == 2 else v.expand(1, -1), want, f"{case}.{k}")
    assert z[f"{case}__qualified_signal"].sum() > 0   # the fixture exercises signals


def test_pump_score_matches_reference(cuda):
    from binquant_amd.strategies import pump_score_features

    z = np.load(G / "liquidation_sweep.npz")
    col = lambda k: torch.from_numpy(z[k])[None].cuda()  # noqa: E731
    t = z["open_time"].astype(np.int64)
    btc = pd.Series(z["btc_close"], index=z["btc_open_time"].astype(np.int64)).reindex(t).to_numpy()
    out = pump_score_features(col("open"), col("high"), col("low"), col("close"), col("volume"),
                              torch.from_numpy(btc).cuda())
    for k, v in out.items():
        _cmp(v, z[k], k)


@pytest.mark.parametrize("stat,window,minp,shift,q", [
    ("median", 19, 19, 2, 0.5), ("median", 20, 5, 0, 0.5), ("quantile", 80, 20, 1, 0.92),
    ("quantile", 48, 48, 1, 0.80), ("max", 6, 6, 1, 1.0), ("min", 6, 6, 1, 0.0),
    ("mean", 20, 20, 1, 0.5), ("sum", 3, 3, 0, 0.5), ("quantile", 96, 1, 0, 0.33),
])
def test_rolling_primitive_vs_pandas(cuda, stat, window, minp, shift, q):
    from binquant_amd import engine
    from binquant_amd.synth import numpy_panel

    S, T = 9, 1300
    x = numpy_panel(S, T, seed0=window + shift, edges=True)["volume"]
    x[:, 100:110] = np.nan   # NaN gaps are skipped (nobs)
    x[2, 500:700] = 3.25     # constant run (same-value rule for mean)
    got = engine.rolling(torch.from_numpy(x).cuda(), window, stat, q=q, min_periods=minp, shift=shift).cpu().numpy()
    for s in range(S):
        r = pd.Series(x[s]).shift(shift).rolling(window, min_periods=minp)
        want = {"median": r.median, "mean": r.mean, "sum": r.sum, "max": r.max, "min": r.min}.get(
            stat, lambda: r.quantile(q))()
        np.testing.assert_allclose(got[s], want.to_numpy(), rtol=1e-12, atol=1e-12, equal_nan=True,
                                   err_msg=f"{stat} row {s}")


@pytest.mark.parametrize("alpha,minp", [(1 / 14, 14), (2 / 21, 0), (0.5, 3)])
def test_ewm_primitive_is_pandas_bitwise(cuda, alpha, minp):
    from binquant_amd import engine

    rng = np.random.default_rng(5)
    x = 100 * np.exp(np.cumsum(rng.normal(0, 0.01, (4, 900)), axis=1))
    x[:, 50:53] = np.nan
    x[1, 0:5] = np.nan
    x[3, 300:400] = x[3, 300]
    got = engine.ewm(torch.from_numpy(x).cuda(), alpha=alpha, min_periods=minp).cpu().numpy()
    for s in range(4):
        want = pd.Series(x[s]).ewm(alpha=alpha, adjust=False, min_periods=minp).mean().to_numpy()
        np.testing.assert_array_equal(got[s], want)
