"""a20: the signal generators' inline helpers on the device vs the
reference's own outputs (tests/golden/signal_helpers.npz: MeanReversionFade
._rsi/_trend_score, RangeBbRsiMeanReversion._compute_adx/_compute_zscore and
TopGainerEarlyMomentum._features evaluated on every prefix frame)."""

from pathlib import Path

import numpy as np
import pytest
import torch

from oracle import indicators_ref
from tests.util import assert_close, assert_close_or_exact

G = Path(__file__).resolve().parent / "golden"
pytestmark = pytest.mark.gpu
CASES = ["sig_a", "sig_b", "sig_c"]


def _load(case):
    z = np.load(G / "signal_helpers.npz")
    col = lambda k: torch.from_numpy(z[f"{case}__{k}"])[None].cuda()  # noqa: E731
    return z, col


def _close(got, want, name):
    scale = np.nanmax(np.abs(want)) if np.isfinite(want).any() else 1.0
    assert_close(got.cpu().numpy().ravel(), want, name, rtol=1e-9, scale=scale)


@pytest.mark.parametrize("exact", [False, True])
@pytest.mark.parametrize("case", CASES)
def test_wilder_rsi_and_trend(cuda, case, exact):
    from binquant_amd import signals

    z, col = _load(case)
    _close(signals.wilder_rsi(col("close"), exact=exact), z[f"{case}__rsi"], f"{case}.rsi")
    _close(signals.trend_score(col("close")), z[f"{case}__trend_score"], f"{case}.trend")


@pytest.mark.parametrize("exact", [False, True])
@pytest.mark.parametrize("case", CASES)
def test_adx_and_zscore(cuda, case, exact):
    from binquant_amd import signals

    z, col = _load(case)
    _close(signals.adx(col("high"), col("low"), col("close"), exact=exact), z[f"{case}__adx"], f"{case}.adx")
    assert_close_or_exact(signals.zscore(col("close"), exact=exact).cpu().numpy().ravel(), z[f"{case}__zscore"],
                          z[f"{case}__close"], 20, indicators_ref.exact_zscore, f"{case}.zscore", max_cases=0 if exact else 8)


@pytest.mark.parametrize("case", CASES)
def test_top_gainer_features(cuda, case):
    from binquant_amd import signals

    z, col = _load(case)
    qv = col("quote_asset_volume") if f"{case}__quote_asset_volume" in z.files else None
    vals, status = signals.top_gainer_features(col("open"), col("high"), col("low"), col("close"),
                                               col("volume"), qv)
    want_status = z[f"{case}__topgainer_status"]
    got_status = np.array([signals.TG_STATUS[int(s)] for s in status[0].cpu().numpy()])
    np.testing.assert_array_equal(got_status, want_status)
    keys = list(z["topgainer_keys"])
    assert tuple(keys) == signals.TG_KEYS
    tg = z[f"{case}__topgainer"]
    for j, k in enumerate(keys):
        _close(vals[k], tg[:, j], f"{case}.{k}")


def test_helpers_batched_equal_rows(cuda):
    """[S, T] panel evaluation equals row-by-row evaluation."""
    from binquant_amd import signals

    z = np.load(G / "signal_helpers.npz")
    T = min(z[f"{c}__close"].size for c in CASES)
    pan = {k: torch.from_numpy(np.stack([z[f"{c}__{k}"][:T] for c in CASES])).cuda()
           for k in ("open", "high", "low", "close", "volume")}
    both = signals.adx(pan["high"], pan["low"], pan["close"]).cpu().numpy()
    rsi = signals.wilder_rsi(pan["close"]).cpu().numpy()
    for r in range(len(CASES)):
        one = signals.adx(pan["high"][r:r + 1], pan["low"][r:r + 1], pan["close"][r:r + 1]).cpu().numpy()
        np.testing.assert_array_equal(both[r], one[0])
        np.testing.assert_array_equal(rsi[r], signals.wilder_rsi(pan["close"][r:r + 1]).cpu().numpy()[0])


@pytest.mark.parametrize("T", [700, 2048, 2049, 5000])
def test_time_parallel_helpers_match_exact_replay(cuda, T):
    """bq_wilder_rsi / bq_zscore / bq_adx (tiles of 2048 candles, carries
    across tiles) vs the bit-exact replay composition (= pandas) on a
    multi-wave panel with per-symbol price scales and constant stretches:
    1e-9 relative; the zscore sign and the RSI 30 / 70 and ADX 25 cuts equal
    away from a 1e-9 band."""
    from binquant_amd import signals
    from binquant_amd.synth import numpy_panel

    p = numpy_panel(70, T, seed0=T)
    d = {k: torch.from_numpy(v).cuda() for k, v in p.items()}
    for name, fast, exact in (
        ("rsi", signals.wilder_rsi(d["close"]), signals.wilder_rsi(d["close"], exact=True)),
        ("adx", signals.adx(d["high"], d["low"], d["close"]), signals.adx(d["high"], d["low"], d["close"], exact=True)),
        ("zscore", signals.zscore(d["close"]), signals.zscore(d["close"], exact=True)),
    ):
        g, w = fast.cpu().numpy(), exact.cpu().numpy()
        scale = 100.0 if name != "zscore" else 1.0
        if name == "zscore":   # nearly constant windows: pandas' drift, arbitrated by the exact value
            assert_close_or_exact(g, w, p["close"], 20, indicators_ref.exact_zscore, name, scale=scale)
        else:
            assert_close(g, w, name, rtol=1e-9, scale=scale)
        cuts = {"rsi": (30.0, 70.0), "adx": (25.0,), "zscore": (0.0,)}[name]
        for c in cuts:
            far = np.abs(w - c) > 1e-9 * np.maximum(np.abs(w), 1.0)
            np.testing.assert_array_equal((g > c)[far], (w > c)[far], err_msg=f"{name} cut {c}")


def _gap_panel(S: int, T: int, seed: int):
    """numpy_panel rows with missing candles (all fields NaN): single gaps,
    a 5-candle gap, a late listing (leading NaN), gaps at the 2048-candle tile
    boundary, a gap in the first window, a row that is all NaN, and a NaN high
    with a valid low (the true range's skip-NaN max covers it)."""
    from binquant_amd.synth import numpy_panel

    p = numpy_panel(S, T, seed0=seed)
    rng = np.random.default_rng(seed)
    gaps = {0: [300], 1: list(range(500, 505)), 2: list(range(0, 150)), 3: [2047, 2048] if T > 2048 else [T - 2],
            4: [5], 5: list(range(T)), 6: [int(x) for x in rng.integers(1, T, 12)], 7: [1, 2, 3],
            8: list(range(0, 20)) + [600]}
    for r, ts in gaps.items():
        for k in ("open", "high", "low", "close", "volume"):
            p[k][r, ts] = np.nan
    p["high"][9, [40, 41, 900 % T]] = np.nan
    return p


@pytest.mark.parametrize("T", [700, 2049, 4100])
def test_time_parallel_helpers_missing_candles(cuda, T):
    """the time-parallel kernels on rows with missing candles
    (NaN gaps, late listings) follow pandas' NaN rules — Wilder RSI against
    pandas' own ewm(adjust=False, ignore_na=False, min_periods) on every row,
    all three against the bit-exact replay composition."""
    import pandas as pd

    from binquant_amd import signals

    p = _gap_panel(70, T, seed=T + 7)
    d = {k: torch.from_numpy(v).cuda() for k, v in p.items()}
    rsi = signals.wilder_rsi(d["close"]).cpu().numpy()
    for r in range(12):
        delta = pd.Series(p["close"][r]).diff()
        ag = delta.clip(lower=0).ewm(alpha=1 / 14, min_periods=14, adjust=False).mean()
        al = (-delta.clip(upper=0)).ewm(alpha=1 / 14, min_periods=14, adjust=False).mean()
        den = ag + al
        want = (100 * ag / den).where(den != 0, 50.0).to_numpy()
        assert_close(rsi[r], want, f"rsi row {r}", rtol=1e-9, scale=100.0)
    for name, fast, exact in (
        ("rsi", rsi, signals.wilder_rsi(d["close"], exact=True).cpu().numpy()),
        ("adx", signals.adx(d["high"], d["low"], d["close"]).cpu().numpy(),
         signals.adx(d["high"], d["low"], d["close"], exact=True).cpu().numpy()),
        ("zscore", signals.zscore(d["close"]).cpu().numpy(), signals.zscore(d["close"], exact=True).cpu().numpy()),
    ):
        if name == "zscore":
            assert_close_or_exact(fast, exact, p["close"], 20, indicators_ref.exact_zscore, name, scale=1.0)
        else:
            assert_close(fast, exact, name, rtol=1e-9, scale=100.0)


@pytest.mark.parametrize("T", [700, 2049])
def test_time_parallel_helpers_other_windows(cuda, T):
    """The kernels are instantiated for the reference's windows (z-score 20,
    ADX 14: the window walks unrolled at compile time); any other window takes
    the generic instantiation — checked here against the exact replay."""
    from binquant_amd import signals
    from binquant_amd.synth import numpy_panel

    p = numpy_panel(70, T, seed0=T + 1)
    d = {k: torch.from_numpy(v).cuda() for k, v in p.items()}
    for w in (10, 33):
        g = signals.adx(d["high"], d["low"], d["close"], window=w).cpu().numpy()
        e = signals.adx(d["high"], d["low"], d["close"], window=w, exact=True).cpu().numpy()
        assert_close(g, e, f"adx{w}", rtol=1e-9, scale=100.0)
        g = signals.zscore(d["close"], window=w).cpu().numpy()
        e = signals.zscore(d["close"], window=w, exact=True).cpu().numpy()
        assert_close_or_exact(g, e, p["close"], w, indicators_ref.exact_zscore, f"zscore{w}", scale=1.0)
