"""CPU: pin the oracle against golden vectors produced by the reference's own
modules (tests/golden/make_golden.py), and the oracle's EWM recursion against
pandas bit for bit."""

import json
from pathlib import Path

import numpy as np
import pandas as pd
import pytest

from oracle import indicators_ref, market_ref

G = Path(__file__).resolve().parent / "golden"


def test_ewm_scalar_is_pandas_bitwise():
    rng = np.random.default_rng(0)
    x = 100 * np.exp(np.cumsum(rng.normal(0, 0.002, 2000)))
    x[300:340] = x[300]
    x[900:905] = np.nan
    for span in (9, 12, 20, 26, 50):
        a = 1.0 / (1.0 + (span - 1) / 2.0)
        want = pd.Series(x).ewm(span=span, adjust=False).mean().to_numpy()
        np.testing.assert_array_equal(indicators_ref.ewm_scalar(x, a), want)


def test_market_features_match_reference_golden():
    z = np.load(G / "market_features.npz")
    cols = list(z["feature_columns"])
    for name in z["names"]:
        name = str(name)
        got = market_ref.symbol_features(z[f"{name}__high"], z[f"{name}__low"], z[f"{name}__close"])
        if bool(z[f"{name}__none"]):
            assert got is None, name
            continue
        want = z[f"{name}__features"]
        vals = np.array([float(got[k]) for k in cols])
        np.testing.assert_array_equal(vals, want, err_msg=name)


def _reference_contexts():
    meta = json.loads((G / "market_context.json").read_text())
    panels = np.load(G / "market_context_panels.npz")
    return meta, panels


@pytest.mark.parametrize("label", ["trend_up_40", "random_64", "selloff_64"])
def test_oracle_context_matches_reference_golden(label):
    meta, panels = _reference_contexts()
    sc = meta[label]
    syms = sc["symbols"]
    ts_all = panels[f"{label}__timestamp"][0]
    h, l, c = (panels[f"{label}__{k}"] for k in ("high", "low", "close"))
    prev = None
    for ts, want in zip(sc["timestamps"], sc["contexts"]):
        t = int(np.flatnonzero(ts_all == ts)[0])
        feats = {}
        for i, s in enumerate(syms):
            f = market_ref.panel_features_at(h[i], l[i], c[i], t, sc["max_bars"])
            if f is not None:
                feats[s] = f
        ctx = market_ref.build_context_from_features(feats, sc["btc"], len(syms), feats.get(sc["btc"]))
        if want is None:
            assert ctx is None
            continue
        ctx["timestamp"] = ts
        ctx = market_ref.annotate_market(ctx, prev)
        for k, v in want.items():
            if k in ("symbol_features", "metadata", "btc_symbol", "confidence", "is_provisional", "timestamp"):
                continue
            if isinstance(v, float):
                assert ctx[k] == pytest.approx(v, rel=1e-12, abs=1e-15), k
            else:
                assert ctx[k] == v, k
        prev = ctx


def test_sma_rsi_matches_reference_helper():
    """pybinbot's rsi column is SMA-smoothed; the in-repo twin is
    BBExtremeReversion._compute_rsi (bb_extreme_reversion.py:134-150)."""
    z = np.load(G / "rsi_helpers.npz")
    for k in ("walk", "rally", "flat", "selloff"):
        c = z[f"{k}__close"]
        df = indicators_ref.rsi(pd.DataFrame({"close": c}))
        ours = df["rsi"].to_numpy()
        want = z[f"{k}__sma_rsi_last"]   # last value of the helper on c[:n+1], clamped
        got = np.clip(ours, 0.0, 100.0)
        m = ~np.isnan(want)
        np.testing.assert_array_equal(np.isnan(got[m]), False, err_msg=k)
        np.testing.assert_allclose(got[m], want[m], rtol=1e-13, atol=1e-12, err_msg=k)
        # the helper refuses fewer than window+1 closes; the column is NaN for < window
        assert np.isnan(ours[:13]).all()


def test_rolling_replays_are_bit_exact_vs_pandas():
    """The step-by-step roll_mean / roll_var restatements that bq_store_features
    replays on the device equal pandas 2.3.3 bit for bit (random walks,
    constant runs, rounded prices, windows 14 and 20, min_periods 1)."""
    from oracle.market_ref import roll_mean_replay, roll_var_replay

    rng = np.random.default_rng(0)
    for trial in range(120):
        n = int(rng.integers(1, 260))
        x = 100 * np.exp(np.cumsum(rng.normal(0, 0.01, n)))
        if trial % 3 == 0:
            k = int(rng.integers(0, n))
            x[k : k + 25] = x[k]
        if trial % 5 == 0:
            x = np.round(x, 2)
        for w in (14, 20):
            s = pd.Series(x).rolling(w, min_periods=1)
            np.testing.assert_array_equal(roll_mean_replay(x, w), s.mean().to_numpy())
            np.testing.assert_array_equal(roll_var_replay(x, w), s.var(ddof=0).to_numpy())


# ---- vectorised oracle forms used by the C3 / C5 size checks --------------------
def test_window_features_equal_per_symbol_features():
    """market_ref.window_features (all symbols at once) == symbol_features per
    symbol, bit for bit, incl. 2-bar windows, constant runs and zero closes."""
    from binquant_amd.synth import numpy_panel

    p = numpy_panel(24, 460, seed0=5)
    p["close"][3, 200:] = p["close"][3, 200]
    p["high"][3, 200:] = p["low"][3, 200:] = p["close"][3, 200]
    p["close"][4, -1] = 0.0
    p["close"][5, -2] = 0.0
    for t, M in ((1, 400), (13, 400), (459, 400), (300, 50), (459, 2)):
        f = market_ref.panel_window_features_at(p["high"], p["low"], p["close"], t, M)
        for s in range(24):
            want = market_ref.panel_features_at(p["high"][s], p["low"][s], p["close"][s], t, M)
            for k in ("return_pct", "ema20", "ema50", "trend_score", "atr_pct", "bb_width", "above_ema20",
                      "above_ema50", "close"):
                assert f[k][s] == want[k] or (np.isnan(f[k][s]) and np.isnan(want[k])), (t, M, s, k)
        assert market_ref.panel_window_features_at(p["high"], p["low"], p["close"], 0, 400) is None


def test_ema_family_panel_equals_per_frame_enrichment():
    from binquant_amd.synth import numpy_panel
    from oracle import indicators_ref as ref

    p = numpy_panel(12, 300, seed0=8)
    p["close"][2, 50] = np.nan   # NaN gap: old weight decays (ignore_na=False)
    p["close"][3, 0] = np.nan    # NaN first value
    want = ref.enrich_panel(p["open"], p["high"], p["low"], p["close"], p["volume"])
    got = ref.ema_family_panel(p["close"])
    for k in ("macd", "macd_signal", "ema20", "ema50"):
        np.testing.assert_array_equal(got[k], want[k], err_msg=k)


def test_strategy_panel_inputs_regenerate_bit_exact():
    """tests/golden/strategy_panel.npz records the reference's outputs for the
    panel_gen inputs; the inputs are regenerated from seeds (digest pinned)."""
    import importlib.util

    spec = importlib.util.spec_from_file_location("panel_gen", Path(__file__).resolve().parent / "golden" / "panel_gen.py")
    pg = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(pg)
    z = np.load(Path(__file__).resolve().parent / "golden" / "strategy_panel.npz")
    assert pg.digest(pg.strategy_panel(*z["positions"].shape[:1], 1100)) == str(z["digest"])
    np.testing.assert_array_equal(pg.sample_positions(64, 1100), z["positions"])


def test_leadership_oracle_equals_reference():
    """oracle.indicators_ref.gradual_gainer_leadership vs the reference's own
    GradualGainerRetest._leadership_allows on every prefix frame
    (tests/golden/leadership.npz: the reference test's make_frames and a
    20 x 360 panel with BTC gaps, a duplicated BTC time and non-positive
    closes): booleans and relative strengths bit-exact."""
    z = np.load(G / "leadership.npz")
    for case in ("ref", "pan"):
        lead, r2, r6 = indicators_ref.gradual_gainer_leadership(
            z[f"{case}__open_time"], z[f"{case}__close"], z[f"{case}__btc_time"], z[f"{case}__btc_close"])
        np.testing.assert_array_equal(lead, z[f"{case}__leader"])
        np.testing.assert_array_equal(r2, z[f"{case}__rs_2h"])
        np.testing.assert_array_equal(r6, z[f"{case}__rs_6h"])
    assert z["ref__leader"][0, -1]   # the reference test's assertion (leader, rs > 0)
