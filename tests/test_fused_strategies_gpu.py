"""The fused strategy passes against the staged pipelines they replace, on
panels with halts, gaps, zero volume and NaN candles:

* bq_pump_features (strategies.pump_score_features, panel mode) — one pass per
  row for every column but the quantiles and score_cross;
* bq_burst_features / bq_burst_qualify (strategies.activity_burst_features)
  — two streaming passes around the score's quantile, bit for bit.

The staged pipelines themselves are pinned to the reference's fixtures
(tests/test_strategies_gpu.py, tests/test_panel_fixtures_gpu.py), which now run
the fused passes too."""

import numpy as np
import pytest
import torch

from tests.util import assert_close

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("ewm_in_pass", [True, False])
def test_pump_fused_equals_staged_panel(cuda, ewm_in_pass, monkeypatch):
    """bq_pump_features (one pass per row) against the staged panel pipeline
    on a 200 x 2500 panel with halts, gaps and zero volume: columns whose
    windows are order statistics / shifts equal bit for bit, the volume mean
    and what depends on it within 1e-12 of each row's magnitude (its sliding
    sum restarts at each lane's 4 candles instead of 8), flags equal away
    from near-ties. With the ewm columns formed in the pass
    (bq_pump_features_ewm: 4-candle lane maps and a DPP scan instead of the
    panel kernel's 8-candle maps) those columns and what depends on them are
    within 1e-12 of the row's magnitude too."""
    from binquant_amd import strategies

    monkeypatch.setattr(strategies, "_PUMP_EWM_IN_PASS", ewm_in_pass)
    from binquant_amd.synth import numpy_panel

    S, T = 200, 2500
    p = numpy_panel(S, T, seed0=31, edges=True)
    p["volume"][3, 700:760] = 0.0
    p["close"][4, 900:905] = np.nan
    d = {k: torch.from_numpy(v).cuda() for k, v in p.items()}
    btc = d["close"][0].clone()
    btc[::17] = float("nan")
    run = lambda: strategies.pump_score_features(d["open"], d["high"], d["low"], d["close"], d["volume"], btc)
    fused = run()
    strategies._PUMP_FUSED = False
    try:
        staged = run()
    finally:
        strategies._PUMP_FUSED = True
    assert list(fused) == list(staged)
    exact_cols = ("candidate_atr", "momentum_3", "pre_breakout_compression", "prior_high", "close_location", "ema20",
                  "ema50", "trend_score", "momentum_atr", "btc_momentum_3", "btc_trend_score", "relative_strength")
    if ewm_in_pass:
        exact_cols = tuple(k for k in exact_cols if k not in ("candidate_atr", "ema20", "ema50", "trend_score",
                                                               "momentum_atr"))
    for k in staged:
        x, y = fused[k].cpu().numpy(), staged[k].cpu().numpy()
        if k in exact_cols:
            np.testing.assert_array_equal(x, y, err_msg=k)
        elif y.dtype == bool:
            assert int((x != y).sum()) <= 5, k
        else:
            with np.errstate(all="ignore"):
                fin = np.where(np.isfinite(y), np.abs(y), np.nan)
                sc = np.nan_to_num(np.nanmax(fin, axis=1, initial=0.0), nan=1.0)
            sc = np.where(sc > 0, sc, 1.0)
            if k == "trend_score":   # (ema20 - ema50) / ema50: the emas' rounding relative to 1, not to the difference
                sc = np.maximum(sc, 1.0)
            assert_close(x, y, f"fused.{k}", rtol=1e-12, scale=np.broadcast_to(sc[:, None], y.shape), atol_rel=1e-13)



@pytest.mark.parametrize("with_q", [True, False])
def test_burst_fused_equals_staged(cuda, with_q):
    from binquant_amd import strategies
    from binquant_amd.synth import numpy_panel

    S, T = 150, 2300
    p = numpy_panel(S, T, seed0=77, edges=True)
    p["volume"][3, 700:760] = 0.0
    p["close"][4, 900:905] = np.nan
    rng = np.random.default_rng(5)
    spikes = rng.random((S, T)) < 0.02   # volume / price bursts so the flags fire
    p["volume"][spikes] *= 8.0
    p["close"][spikes] *= 1.03
    p["high"] = np.fmax(p["high"], p["close"])
    d = {k: torch.from_numpy(v).cuda() for k, v in p.items()}
    qv = d["volume"] * d["close"] if with_q else None
    run = lambda: strategies.activity_burst_features(d["open"], d["high"], d["low"], d["close"], d["volume"], qv)
    fused = run()
    strategies._BURST_FUSED = False
    try:
        staged = run()
    finally:
        strategies._BURST_FUSED = True
    assert list(fused) == list(staged)
    for k in staged:
        x, y = fused[k].cpu().numpy(), staged[k].cpu().numpy()
        assert x.dtype == y.dtype, k
        np.testing.assert_array_equal(x, y, err_msg=k)
    assert staged["qualified_signal"].sum().item() > 0


def test_spike_fused_equals_staged(cuda):
    """bq_spike_base(_std) / bq_spike_flags against the staged failed-spike
    pipeline (panel mode): everything computed from raw values (geometry, pct
    changes, momentum, integer counts, streak flags) equal bit for bit; the
    rolling means / sums (direct window sums here, sliding in the staged panel
    kernel) and their dependants within 1e-12 of each row's magnitude; the five
    std columns (formed in the base pass by default, the staged pipeline's
    replays of pandas' online variance) and their descendants by
    tests/spike_std.py's rule (1e-9, or closer to the exact window std where
    pandas drifts); flags equal away from near-ties of their thresholds (a
    handful at most)."""
    from binquant_amd import strategies
    from binquant_amd.synth import numpy_panel

    S, T = 160, 2200
    p = numpy_panel(S, T, seed0=91, edges=True)
    p["volume"][3, 700:760] = 0.0
    p["close"][4, 900:905] = np.nan
    rng = np.random.default_rng(8)
    spikes = rng.random((S, T)) < 0.02
    p["volume"][spikes] *= 6.0
    p["close"][spikes] *= 1.04
    p["high"] = np.fmax(p["high"], p["close"])
    d = {k: torch.from_numpy(v).cuda() for k, v in p.items()}
    qv = d["volume"] * d["close"]
    run = lambda: strategies.failed_spike_features(d["open"], d["high"], d["low"], d["close"], d["volume"], qv)
    fused = run()
    strategies._SPIKE_FUSED = False
    try:
        staged = run()
    finally:
        strategies._SPIKE_FUSED = True
    assert list(fused) == list(staged)
    exact = {"price_change", "price_change_abs", "body_size", "body_size_pct", "upper_wick", "lower_wick",
             "upper_wick_ratio", "lower_wick_ratio", "total_range", "range_pct", "is_bullish", "close_open_ratio",
             "momentum_3", "momentum_5", "close_to_high", "close_to_low", "pc_1", "pc_pos_count_5",
             "upward", "downward", "early_spike_proba", "early_proba_aug_flag"}
    from tests import spike_std

    fn_, sn_ = ({k: v.cpu().numpy() for k, v in m.items()} for m in (fused, staged))
    spike_std.check(fn_, sn_, {"close": p["close"], "volume": p["volume"], "body_size_pct": sn_["body_size_pct"]})
    if not strategies._SPIKE_STD_IN_PASS:   # the replays on both sides: bit for bit
        exact |= set(spike_std.STD_COLS) | {"std_ratio_8_20", "vol_compression_flag"}
    flips = 0
    for k in staged:
        x, y = fused[k].cpu().numpy(), staged[k].cpu().numpy()
        assert x.dtype == y.dtype and x.shape == y.shape, k
        if k in exact:
            np.testing.assert_array_equal(x, y, err_msg=k)
        elif k in spike_std.STD_COLS or k in spike_std.DESC:
            continue   # checked by spike_std.check (1e-9, or explained by pandas' drift)
        elif y.dtype == bool:
            flips += int((x != y).sum())
        else:
            x2, y2 = (x[:, None], y[:, None]) if y.ndim == 1 else (x, y)
            with np.errstate(all="ignore"):
                fin = np.where(np.isfinite(y2), np.abs(y2), np.nan)
                sc = np.nan_to_num(np.nanmax(fin, axis=1, initial=0.0), nan=1.0)
            sc = np.where(sc > 0, sc, 1.0)
            assert_close(x2, y2, f"fused.{k}", rtol=1e-12, scale=np.broadcast_to(sc[:, None], y2.shape),
                         atol_rel=1e-13)
    assert flips <= 10, flips
    assert staged["label"].sum().item() > 0


@pytest.mark.parametrize("S,T", [(7, 1001), (3, 5), (1, 1025), (5, 2), (6, 4500)])
def test_fused_odd_shapes_equal_staged(cuda, S, T):
    """Odd T (rows not 16-byte aligned: the scalar load / store paths, byte
    flags unaligned), tiny rows and a partial second tile: the three fused
    paths against their staged pipelines — burst bit for bit, pump / spike to
    1e-12 / the z-score bound as above, flags equal. At T = 4500, halted
    stretches (constant price, zero volume) and a NaN stretch cross the 1024 /
    2048 / 4096-candle tile boundaries, so every cross-tile carry (volume run
    start, ffill index, ring halo) is exercised."""
    from binquant_amd import engine, strategies
    from binquant_amd.synth import numpy_panel

    p = numpy_panel(S, T, seed0=S * 100 + T, edges=T > 50)
    if T > 4150:
        for s, (a, b) in enumerate(((1010, 1040), (2030, 2100), (4080, 4150))):
            for f in ("open", "high", "low", "close"):
                p[f][s, a:b] = p["close"][s, a]
            p["volume"][s, a:b] = 0.0
            p["volume"][s + 3, a:b] = 0.0
        p["close"][5, 2040:2056] = np.nan
    d = {k: torch.from_numpy(v).cuda() for k, v in p.items()}
    qv = d["volume"] * d["close"]
    btc = d["close"][0].clone()
    calls = {
        "burst": (lambda: strategies.activity_burst_features(d["open"], d["high"], d["low"], d["close"], d["volume"],
                                                             qv), "_BURST_FUSED"),
        "pump": (lambda: strategies.pump_score_features(d["open"], d["high"], d["low"], d["close"], d["volume"], btc),
                 "_PUMP_FUSED"),
        "spike": (lambda: strategies.failed_spike_features(d["open"], d["high"], d["low"], d["close"], d["volume"], qv),
                  "_SPIKE_FUSED"),
    }
    for name, (fn, flag) in calls.items():
        fused = fn()
        setattr(strategies, flag, False)
        try:
            staged = fn()
        finally:
            setattr(strategies, flag, True)
        assert list(fused) == list(staged), name
        if name == "spike":   # the std columns and their descendants: tests/spike_std.py's rule
            from tests import spike_std

            fn_, sn_ = ({k: v.cpu().numpy() for k, v in m.items()} for m in (fused, staged))
            spike_std.check(fn_, sn_, {"close": p["close"], "volume": p["volume"], "body_size_pct": sn_["body_size_pct"]})
        for k in staged:
            x, y = fused[k].cpu().numpy(), staged[k].cpu().numpy()
            assert x.dtype == y.dtype and x.shape == y.shape, (name, k)
            if name == "spike" and (k in spike_std.STD_COLS or k in spike_std.DESC):
                continue   # spike_std.check (1e-9, or explained by pandas' drift)
            if y.dtype == bool or name == "burst":
                np.testing.assert_array_equal(x, y, err_msg=f"{name}.{k}")
                continue
            np.testing.assert_array_equal(np.isnan(x), np.isnan(y), err_msg=f"{name}.{k}")
            with np.errstate(all="ignore"):
                y2 = y if y.ndim == 2 else y[:, None]
                fin = np.where(np.isfinite(y2), np.abs(y2), np.nan)
                sc = np.nan_to_num(np.nanmax(fin, axis=1, initial=0.0), nan=1.0)
                sc = np.where(sc > 0, sc, 1.0)
                lim = 1e-12 * np.abs(y) + 1e-13 * (sc[:, None] if y.ndim == 2 else sc)
                if name == "pump" and k == "trend_score":   # the emas' rounding relative to 1 (cancellation)
                    lim = lim + 1e-13
                ok = np.isnan(y) | (x == y) | (np.abs(x - y) <= lim)   # x == y: equal infinities (v / 0)
            assert ok.all(), (name, k, int((~ok).sum()))


@pytest.mark.parametrize("S,T", [(9, 3100), (4, 3), (3, 1024), (2, 1)])
def test_pump_ewm_in_pass_against_pandas(cuda, S, T):
    """bq_pump_features_ewm's candidate_atr / ema20 / ema50 (the scans inside
    the pass, pandas' recursion from the first tile holding a missing or
    infinite value) against pandas' ewm (adjust=False) of the true range /
    close and against bq_pump_ewm, at 1e-12 of each row's magnitude with the
    NaN positions equal: a late listing (leading NaNs past the first tile), a
    NaN high only (the true range alone turns serial), an infinite close, a
    NaN first candle, a NaN stretch across a tile boundary, an all-NaN row."""
    import pandas as pd

    from binquant_amd import engine
    from binquant_amd.synth import numpy_panel

    p = numpy_panel(S, T, seed0=7 * S + T, edges=False)
    h, l, c, v = (p[k].copy() for k in ("high", "low", "close", "volume"))
    if T > 3000:
        h[0, :] = l[0, :] = c[0, :] = np.nan
        h[1, :1500] = l[1, :1500] = c[1, :1500] = np.nan
        h[2, 700] = np.nan
        c[3, 2000] = np.inf
        h[4, 0] = l[4, 0] = c[4, 0] = np.nan
        c[5, 1020:1030] = np.nan
        h[6, 2040:2060] = l[6, 2040:2060] = np.nan
    d = [torch.from_numpy(x).cuda() for x in (h, l, c, v)]
    bench = torch.from_numpy(c[-1].copy()).cuda()
    got = engine.pump_features_ewm(*d, bench, bench, bench)
    ref = engine.pump_ewm(d[0], d[1], d[2])
    for r in range(S):
        hs, ls, cs = pd.Series(h[r]), pd.Series(l[r]), pd.Series(c[r])
        tr = pd.concat([hs - ls, (hs - cs.shift(1)).abs(), (ls - cs.shift(1)).abs()], axis=1).max(axis=1)
        want = {"candidate_atr": tr.ewm(alpha=1 / 14, adjust=False, min_periods=14).mean().to_numpy(),
                "ema20": cs.ewm(span=20, adjust=False).mean().to_numpy(),
                "ema50": cs.ewm(span=50, adjust=False).mean().to_numpy()}
        for i, k in enumerate(("candidate_atr", "ema20", "ema50")):
            x = got[k][r].cpu().numpy()
            for name, y in ((f"pandas {k} row {r}", want[k]), (f"bq_pump_ewm {k} row {r}", ref[i][r].cpu().numpy())):
                np.testing.assert_array_equal(np.isnan(x), np.isnan(y), err_msg=name)
                fin = np.isfinite(y)
                np.testing.assert_array_equal(x[~fin & ~np.isnan(y)], y[~fin & ~np.isnan(y)], err_msg=name)
                sc = float(np.max(np.abs(y[fin]))) if fin.any() else 1.0
                assert np.all(np.abs(x[fin] - y[fin]) <= 1e-12 * np.abs(y[fin]) + 1e-13 * sc), name


@pytest.mark.parametrize("S,T", [(9, 3100), (5, 2048), (3, 7), (2, 1), (3, 2049), (1, 4100)])
def test_pump_ewm_one_pass_equals_panel_ewm(cuda, S, T):
    """bq_pump_ewm's one-pass kernel (the three series on the same tiles)
    against the generic panel ewm (bq_rolling_batch, panel mode) bit for bit
    — ema20 / ema50 of close and the ATR of the true range — including rows
    that turn serial in one series only (a NaN high: the true range; an
    infinite close: both emas; a late listing), and trend_score bit-equal to
    the staged (ema20 - ema50) / ema50."""
    from binquant_amd import engine
    from binquant_amd.synth import numpy_panel

    E = engine.Ewm
    p = numpy_panel(S, T, seed0=3 * S + T, edges=False)
    h, l, c = (p[k].copy() for k in ("high", "low", "close"))
    if T > 3000 and S >= 4:
        h[0, 700] = np.nan
        c[1, 2100] = np.inf
        h[2, :2500] = l[2, :2500] = c[2, :2500] = np.nan
        c[3, 10:20] = np.nan
    d = [torch.from_numpy(x).cuda() for x in (h, l, c)]
    atr, e20, e50, trend = engine.pump_ewm(*d, trend=True)
    pc = np.concatenate([np.full((S, 1), np.nan), c[:, :-1]], axis=1)
    tr = np.fmax(np.fmax(h - l, np.abs(h - pc)), np.abs(l - pc))
    w_atr, w20, w50 = engine.rolling_many(E(torch.from_numpy(tr).cuda(), alpha=1 / 14, min_periods=14),
                                          E(d[2], span=20), E(d[2], span=50), exact=False)
    for name, x, y in (("atr", atr, w_atr), ("ema20", e20, w20), ("ema50", e50, w50)):
        np.testing.assert_array_equal(x.cpu().numpy(), y.cpu().numpy(), err_msg=name)
    np.testing.assert_array_equal(trend.cpu().numpy(), ((e20 - e50) / e50).cpu().numpy())
    a3 = engine.pump_ewm(*d)
    assert len(a3) == 3
    for x, y in zip(a3, (atr, e20, e50)):
        np.testing.assert_array_equal(x.cpu().numpy(), y.cpu().numpy())


@pytest.mark.parametrize("S,T,w,q", [(2100, 2000, 48, 0.80), (2100, 2000, 80, 0.92), (40, 700, 48, 0.80),
                                     (2100, 2000, 30, 0.5)])
def test_rolling_quantile_cross(cuda, S, T, w, q):
    """bq_rolling_quantile_cross: the threshold bit-equal to bq_rolling's
    quantile of x.shift(1) (the sliding-window kernel at large panels, with
    the flags formed in its steps and the window of each segment's previous
    step built for the first flag; the tile / stencil kernels + a flag pass
    elsewhere) and cross = (x >= thr) & (x.shift(1) < thr.shift(1)) bit for
    bit, on rows with NaN runs, a constant stretch and a late start."""
    from binquant_amd import engine
    from binquant_amd.synth import numpy_panel

    x = numpy_panel(S, T, seed0=S + w, edges=False)["volume"].copy()
    x[1, 300:340] = np.nan
    x[2, :500] = np.nan
    x[3, 100:400] = 5.0
    x[4, ::7] = np.nan
    d = torch.from_numpy(x).cuda()
    thr, cross = engine.rolling_quantile_cross(d, w, q, shift=1)
    want = engine.rolling(d, w, "quantile", q=q, shift=1)
    np.testing.assert_array_equal(thr.cpu().numpy(), want.cpu().numpy())
    t = want.cpu().numpy()
    with np.errstate(invalid="ignore"):
        c = (x >= t) & np.concatenate([np.zeros((S, 1), bool), x[:, :-1] < t[:, :-1]], axis=1)
    got = cross.cpu().numpy()
    assert got.dtype == bool
    np.testing.assert_array_equal(got, c)
    assert c.sum() > 0
    # in a batch beside a quantile without flags (one launch of the flag
    # instantiation where the slide kernel runs), flags on the second spec
    d2 = torch.flip(d, dims=[1]).contiguous()
    (a, b), (f,) = engine.rolling_many(engine.Roll(d2, w, "quantile", q=q, shift=1),
                                       engine.Roll(d, w, "quantile", q=q, shift=1), exact=False, cross=(1,))
    np.testing.assert_array_equal(b.cpu().numpy(), t)
    np.testing.assert_array_equal(a.cpu().numpy(), engine.rolling(d2, w, "quantile", q=q, shift=1).cpu().numpy())
    np.testing.assert_array_equal(f.cpu().numpy(), c)
