"""a17/a18/a19: strategy feature pipelines (bq_rolling / bq_ewm / bq_select
kernels + device glue) vs the reference's own outputs
(tests/golden/activity_burst.npz, liquidation_sweep.npz, failed_spike.npz from
strategies/activity_burst_pump.py:51-158, strategies/liquidation_sweep_pump.py:195-269
and strategies/failed_spike_fade.py:533-544), and the primitives vs pandas /
numpy / the reference's cooldown loop on larger panels."""

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
    ("var", 12, 12, 0, 0.5), ("std", 20, 20, 0, 0.5), ("std", 8, 2, 1, 0.5), ("sum", 8, 0, 0, 0.5),
    ("sum", 8, 1, 0, 0.5), ("mean", 10, 3, 2, 0.5),
])
def test_rolling_primitive_vs_pandas(cuda, stat, window, minp, shift, q):
    from binquant_amd import engine
    from binquant_amd.synth import numpy_panel

    S, T = 70, 1300   # 70 rows: a full and a partial wave of the lane-per-symbol replay
    x = numpy_panel(S, T, seed0=window + shift, edges=True)["volume"]
    x[:, 100:110] = np.nan   # NaN gaps are skipped (nobs)
    x[2, 500:700] = 3.25     # constant run (same-value rule for mean)
    got = engine.rolling(torch.from_numpy(x).cuda(), window, stat, q=q, min_periods=minp, shift=shift).cpu().numpy()
    for s in range(S):
        r = pd.Series(x[s]).shift(shift).rolling(window, min_periods=minp)
        want = {"median": r.median, "mean": r.mean, "sum": r.sum, "max": r.max, "min": r.min,
                "var": r.var, "std": r.std}.get(stat, lambda: r.quantile(q))()
        # bit-exact: moments replay pandas' recurrences, order statistics are exact
        np.testing.assert_array_equal(got[s], want.to_numpy(), err_msg=f"{stat} row {s}")


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


@pytest.mark.parametrize("stat,window,minp", [("sum", 3, 3), ("sum", 2, 2), ("mean", 10, 10), ("std", 10, 10),
                                              ("var", 12, 3)])
def test_rolling_signed_series_vs_pandas(cuda, stat, window, minp):
    """Signed inputs (price changes) exercise the mean sign clamps and the
    compensated sums."""
    from binquant_amd import engine

    rng = np.random.default_rng(window)
    x = rng.normal(0, 0.01, (6, 2000))
    x[0, :] = np.abs(x[0, :])
    x[1, :] = -np.abs(x[1, :])
    x[2, 40:44] = np.nan
    x[3, 600:900] = -0.0125
    x[4, 1000:1300] = 0.0
    got = engine.rolling(torch.from_numpy(x).cuda(), window, stat, min_periods=minp).cpu().numpy()
    for s in range(6):
        r = pd.Series(x[s]).rolling(window, min_periods=minp)
        want = getattr(r, stat)().to_numpy()
        np.testing.assert_array_equal(got[s], want, err_msg=f"{stat} {s}")


# register-resident row forms: a wave per row (T <= 2048), a workgroup per row (8 / 16 / 40 keys per thread)
@pytest.mark.parametrize("T", [200, 700, 2000, 2048, 3000, 9000])
def test_row_quantile_is_numpy_bitwise(cuda, T):
    from binquant_amd import engine

    rng = np.random.default_rng(11)
    x = rng.lognormal(0, 1, (10, T))
    x[1] = rng.normal(0, 1, T)                    # negatives
    x[2] = np.round(rng.normal(0, 3, T))          # heavy ties
    x[3, :] = np.nan                              # empty row
    x[4, :] = np.nan
    x[4, 17] = 2.5                                # single observation
    x[5, :] = np.nan
    x[5, [3, T - 100]] = [4.0, -1.0]              # two observations
    x[6, ::3] = np.nan                            # ragged NaNs
    x[7, :] = 7.0                                 # constant
    x[8, :11] = np.nan                            # leading NaNs (rolling warm-up)
    x[9] = -x[9]
    zeros = np.abs(rng.normal(0, 1e-3, (2, T)))                   # |pct change|: halted candles' exact zeros
    zeros[0, rng.random(T) < 0.4] = 0.0
    zeros[1, rng.random(T) < 0.2] = -0.0
    infs = rng.lognormal(0, 1, (1, T))
    infs[0, rng.random(T) < 0.05] = np.inf
    infs[0, rng.random(T) < 0.05] = -np.inf
    x = np.vstack([x, zeros, infs])
    xt = torch.from_numpy(x).cuda()
    for q in (0.0, 0.25, 0.5, 0.75, 0.85, 0.97, 1.0, 0.333):
        got = engine.row_quantile(xt, q).cpu().numpy()
        for s in range(x.shape[0]):
            v = x[s][~np.isnan(x[s])]
            with np.errstate(invalid="ignore"):
                want = np.quantile(v, q) if v.size else np.nan
            np.testing.assert_array_equal(got[s], want, err_msg=f"q={q} row {s}")


def test_row_quantile_strided_rows(cuda):
    """Rows of a padded buffer (row stride > T, as enrich_outputs lays them
    out) give the contiguous rows' quantiles bit for bit."""
    from binquant_amd import engine

    rng = np.random.default_rng(13)
    for T in (700, 2000):
        x = rng.lognormal(0, 1, (37, T))
        x[rng.random(x.shape) < 0.05] = np.nan
        buf = torch.full((37, T + 40), 1e300, dtype=torch.float64, device="cuda")
        buf[:, :T] = torch.from_numpy(x).cuda()
        for q in (0.75, 0.97):
            got = engine.row_quantile(buf[:, :T], q).cpu().numpy()
            want = engine.row_quantile(torch.from_numpy(x).cuda(), q).cpu().numpy()
            np.testing.assert_array_equal(got, want)


def test_row_quantile_large_rows(cuda):
    from binquant_amd import engine

    rng = np.random.default_rng(12)
    x = rng.lognormal(0, 2, (64, 20000))
    x[rng.random(x.shape) < 0.01] = np.nan
    got = engine.row_quantile(torch.from_numpy(x).cuda(), 0.97).cpu().numpy()
    want = np.array([np.quantile(r[~np.isnan(r)], 0.97) for r in x])
    np.testing.assert_array_equal(got, want)


def _cooldown_loop(label, bars):
    """strategies/failed_spike_fade.py:504-518 over one row."""
    kept, sup = label.copy(), np.zeros_like(label)
    last = None
    for i in range(label.size):
        if kept[i] == 1:
            if last is not None and (i - last) <= bars:
                sup[i] = 1
                kept[i] = 0
            else:
                last = i
    return kept, sup


@pytest.mark.parametrize("bars", [0, 1, 8, 30])
def test_cooldown_matches_reference_loop(cuda, bars):
    from binquant_amd import engine

    rng = np.random.default_rng(bars)
    lab = rng.random((300, 700)) < 0.15
    lab[0] = True
    lab[1] = False
    kept, sup = engine.cooldown(torch.from_numpy(lab).cuda(), bars)
    kept, sup = kept.cpu().numpy(), sup.cpu().numpy()
    for s in range(lab.shape[0]):
        k, u = _cooldown_loop(lab[s].astype(int), bars)
        np.testing.assert_array_equal(kept[s], k.astype(bool), err_msg=f"row {s}")
        np.testing.assert_array_equal(sup[s], u.astype(bool), err_msg=f"row {s}")


@pytest.mark.parametrize("case", ["fsf_a", "fsf_b", "fsf_c"])
def test_failed_spike_matches_reference(cuda, case):
    from binquant_amd.strategies import failed_spike_features

    z = np.load(G / "failed_spike.npz")
    col = lambda k: torch.from_numpy(z[f"{case}__{k}"])[None].cuda()  # noqa: E731
    out = failed_spike_features(col("open"), col("high"), col("low"), col("close"), col("volume"),
                                col("quote_asset_volume"))
    vcmr, pbbt = z[f"{case}__calibrated"]
    np.testing.assert_allclose(out.pop("volume_cluster_min_ratio").item(), vcmr, rtol=1e-12)
    np.testing.assert_allclose(out.pop("price_break_base_threshold").item(), pbbt, rtol=1e-12)
    golden = {k.split("__", 1)[1] for k in z.files if k.startswith(case + "__")} - {"calibrated"}
    inputs = {"open", "high", "low", "close", "volume", "quote_asset_volume"}
    assert golden - inputs == set(out), sorted((golden - inputs) ^ set(out))
    for k, v in out.items():
        _cmp(v, z[f"{case}__{k}"], f"{case}.{k}")
    assert z[f"{case}__label"].sum() > 0


def test_failed_spike_panel_equals_rows(cuda):
    """Batched [S, T] evaluation equals per-symbol evaluation (no cross-row
    leakage in the per-row calibration, cooldown or rolling kernels)."""
    from binquant_amd.strategies import failed_spike_features

    z = np.load(G / "failed_spike.npz")
    cols = ["open", "high", "low", "close", "volume", "quote_asset_volume"]
    panel = [torch.from_numpy(np.stack([z[f"fsf_a__{k}"], z[f"fsf_b__{k}"]])).cuda() for k in cols]
    both = failed_spike_features(*panel)
    for r, case in enumerate(["fsf_a", "fsf_b"]):
        one = failed_spike_features(*[torch.from_numpy(z[f"{case}__{k}"])[None].cuda() for k in cols])
        for k, v in one.items():
            a, b = both[k][r].cpu().numpy(), v[0].cpu().numpy() if v.dim() == 2 else v.cpu().numpy()[0]
            np.testing.assert_array_equal(a, b, err_msg=f"{case}.{k}")


@pytest.mark.parametrize("S,T", [(37, 700), (300, 2100)])
def test_integer_sum_matches_replayed_sum_bitwise(cuda, S, T):
    """BQ_ROLL_ISUM (a direct window sum for integer-valued series) gives the
    replayed pandas roll_sum bit for bit — signs of zero (pandas' same-value
    rule), NaN gaps, min_periods 0 / 1 / w, shifts, and the long-window
    fallback to the replay — and equals pandas on a sample."""
    from binquant_amd import engine
    from binquant_amd.engine import Roll

    g = torch.Generator().manual_seed(21)
    flags = (torch.rand(S, T, generator=g) < 0.4).double()
    ints = torch.round(torch.randn(S, T, generator=g, dtype=torch.float64) * 3)
    ints[torch.rand(S, T, generator=g) < 0.05] = float("nan")
    ints[0, ::2] = -0.0
    ints[1, 100:180] = -0.0                      # a run of negative zeros
    ints[2, 40:90] = 0.0
    ints[2, 60] = -0.0                           # mixed-sign zero run
    ints[3, :] = float("nan")
    jobs = [(3, 3, 0), (5, 5, 0), (12, 1, 0), (12, 0, 2), (19, 7, 1), (32, 32, 0), (40, 1, 0)]
    for x in (flags.cuda(), ints.cuda()):
        got = engine.rolling_many(*[Roll(x, w, "isum", min_periods=mp, shift=sh) for w, mp, sh in jobs])
        want = engine.rolling_many(*[Roll(x, w, "sum", min_periods=mp, shift=sh) for w, mp, sh in jobs])
        for (w, mp, sh), a, b in zip(jobs, got, want):
            a, b = a.cpu().numpy(), b.cpu().numpy()
            np.testing.assert_array_equal(a, b, err_msg=f"isum w={w} mp={mp} sh={sh}")
            num = ~np.isnan(b)
            assert np.array_equal(np.signbit(a[num]), np.signbit(b[num])), (w, mp, sh)
        xs = x[:4].cpu().numpy()
        for (w, mp, sh), a in zip(jobs, got):
            ref = pd.DataFrame(xs.T).shift(sh).rolling(w, min_periods=mp).sum().to_numpy().T
            np.testing.assert_array_equal(a[:4].cpu().numpy(), ref, err_msg=f"pandas w={w}")


def test_plan_cache_hits_are_bit_exact(cuda):
    """Eager pipelines reuse cached fused plans (binquant_amd.fused plan
    cache): a second panel of the same shape hits the cache (data-dependent
    constants, if any, are new keys), and every output
    equals the same call with the cache disabled, bit for bit."""
    from binquant_amd import fused as F
    from binquant_amd import signals, strategies
    from binquant_amd.synth import device_panel

    # (the staged burst, pump and spike pipelines: their fused paths,
    # bq_burst_features, bq_pump_features + bq_rolling_quantile_cross and
    # bq_spike_base_std + bq_spike_flags, run no JIT programs)
    calls = {
        "burst": lambda o, h, l, c, v: _staged_burst(strategies, o, h, l, c, v),
        "spike": lambda o, h, l, c, v: _staged_spike(strategies, o, h, l, c, v),
        "pump": lambda o, h, l, c, v: _staged_pump(strategies, o, h, l, c, v),
        "gainer": lambda o, h, l, c, v: signals.top_gainer_features(o, h, l, c, v, v * c),
    }
    for seed, (name, fn) in enumerate(calls.items()):
        p = device_panel(48, 300, seed=seed)
        args = [p[k] for k in ("open", "high", "low", "close", "volume")]
        fn(*args)   # populates the cache
        before = F.plan_cache_stats()
        p2 = device_panel(48, 300, seed=seed + 100)
        args2 = [p2[k] for k in ("open", "high", "low", "close", "volume")]
        hot = fn(*args2)
        after = F.plan_cache_stats()
        assert after["hits"] > before["hits"], name
        F._PLAN_CACHE_ON = False
        try:
            cold = fn(*args2)
        finally:
            F._PLAN_CACHE_ON = True
        _assert_same_tree(hot, cold, name)


def _staged_spike(strategies, o, h, l, c, v):
    strategies._SPIKE_FUSED = False
    try:
        return strategies.failed_spike_features(o, h, l, c, v, v * c)
    finally:
        strategies._SPIKE_FUSED = True


def _staged_burst(strategies, o, h, l, c, v):
    strategies._BURST_FUSED = False
    try:
        return strategies.activity_burst_features(o, h, l, c, v, v * c)
    finally:
        strategies._BURST_FUSED = True


def _staged_pump(strategies, o, h, l, c, v):
    strategies._PUMP_FUSED = False
    try:
        return strategies.pump_score_features(o, h, l, c, v, c[0].clone())
    finally:
        strategies._PUMP_FUSED = True


def _assert_same_tree(a, b, path):
    if isinstance(b, dict):
        assert isinstance(a, dict) and set(a) == set(b), path
        for k in b:
            _assert_same_tree(a[k], b[k], f"{path}.{k}")
    elif isinstance(b, (tuple, list)):
        assert len(a) == len(b), path
        for i, (x, y) in enumerate(zip(a, b)):
            _assert_same_tree(x, y, f"{path}[{i}]")
    else:
        x, y = a.cpu().numpy(), b.cpu().numpy()
        assert x.dtype == y.dtype, path
        np.testing.assert_array_equal(x, y, err_msg=path)
