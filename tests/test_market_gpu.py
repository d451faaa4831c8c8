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


# ---- against the reference's own golden vectors ---------------------------------
import json  # noqa: E402
from pathlib import Path  # noqa: E402

from binquant_amd.market_regime.regime import annotate_market, score_contexts  # noqa: E402

G = Path(__file__).resolve().parent / "golden"


def test_features_kernel_matches_reference_golden(cuda):
    z = np.load(G / "market_features.npz")
    cols = [str(c) for c in z["feature_columns"]]
    for name in z["names"]:
        name = str(name)
        h, l, c = (torch.from_numpy(np.ascontiguousarray(z[f"{name}__{k}"]))[None].cuda() for k in ("high", "low", "close"))
        f = engine.market_features(h, l, c, max_bars=400)
        got = {k: float(v[0, -1]) for k, v in f.items()}
        if bool(z[f"{name}__none"]):
            assert all(np.isnan(v) for v in got.values()), name
            continue
        want = dict(zip(cols, z[f"{name}__features"]))
        for k in ("return_pct", "ema20", "ema50", "trend_score", "atr_pct", "bb_width"):
            assert_close([got[k]], [want[k]], f"{name}.{k}", scale=[abs(want["close"]) * 1e-2 + 1e-300])
        assert (want["close"] > got["ema20"]) == bool(want["above_ema20"]), name
        assert (want["close"] > got["ema50"]) == bool(want["above_ema50"]), name


@pytest.mark.parametrize("label", ["trend_up_40", "random_64", "selloff_64"])
def test_device_context_pipeline_matches_reference_golden(cuda, label):
    meta = json.loads((G / "market_context.json").read_text())
    panels = np.load(G / "market_context_panels.npz")
    sc = meta[label]
    syms = sc["symbols"]
    ts_all = panels[f"{label}__timestamp"][0]
    h, l, c = (torch.from_numpy(panels[f"{label}__{k}"]).cuda() for k in ("high", "low", "close"))
    f = engine.market_features(h, l, c, max_bars=sc["max_bars"])
    part = engine.breadth_partial(c, f).cpu().numpy()
    b = syms.index(sc["btc"])
    btc_ret = f["return_pct"][b].cpu().numpy()
    btc_trend = f["trend_score"][b].cpu().numpy()
    idx = [int(np.flatnonzero(ts_all == ts)[0]) for ts in sc["timestamps"]]
    ok = ~np.isnan(btc_ret[idx])
    batch = score_contexts(part[idx], np.nan_to_num(btc_ret[idx]), np.nan_to_num(btc_trend[idx]), ok,
                           total_tracked=len(syms), timestamps=np.array(sc["timestamps"]))
    annotate_market(batch)
    for i, want in enumerate(sc["contexts"]):
        got = batch.context_at(i)
        if want is None:
            assert got is None
            continue
        for k, v in want.items():
            if k in ("symbol_features", "metadata", "btc_symbol", "confidence", "is_provisional", "timestamp"):
                continue
            if isinstance(v, (bool, str, int)) or v is None:
                assert got[k] == v, (k, got[k], v)
            else:
                assert got[k] == pytest.approx(v, rel=1e-9, abs=1e-12), k


@pytest.mark.parametrize("S,T", [(10_000, 1), (3000, 3), (1500, 256), (1500, 257), (5, 1)])
def test_breadth_partial_few_timestamps(cuda, S, T):
    """The few-timestamp path (T <= 256: one workgroup per timestamp, the live
    tick's T = 1) and the boundary to the lane-per-timestamp path: counts
    exact, sums within 1e-12 of numpy, NaN-return rows skipped, bitwise
    reproducible run to run."""
    g = np.random.default_rng(S + T)
    c = g.uniform(1, 100, (S, T))
    fn = {k: g.normal(0, 1, (S, T)) for k in FEATURE_COLUMNS}
    fn["ema20"], fn["ema50"] = c * g.uniform(0.9, 1.1, (S, T)), c * g.uniform(0.9, 1.1, (S, T))
    fn["return_pct"][g.random((S, T)) < 0.1] = np.nan
    fn["return_pct"][:, 0][:3] = 0.0   # neither advancer nor decliner
    f = {k: torch.from_numpy(v).cuda() for k, v in fn.items()}
    part = engine.breadth_partial(torch.from_numpy(c).cuda(), f).cpu().numpy()
    valid = ~np.isnan(fn["return_pct"])
    np.testing.assert_array_equal(part[:, 0], valid.sum(axis=0))
    np.testing.assert_array_equal(part[:, 1], (valid & (fn["return_pct"] > 0)).sum(axis=0))
    np.testing.assert_array_equal(part[:, 2], (valid & (fn["return_pct"] < 0)).sum(axis=0))
    np.testing.assert_array_equal(part[:, 3], (valid & (c > fn["ema20"])).sum(axis=0))
    np.testing.assert_array_equal(part[:, 4], (valid & (c > fn["ema50"])).sum(axis=0))
    for i, k in ((5, "return_pct"), (6, "trend_score"), (7, "atr_pct"), (8, "bb_width")):
        want = np.where(valid, fn[k], 0.0).sum(axis=0)
        assert_close(part[:, i], want, k, rtol=1e-12, scale=np.abs(np.where(valid, fn[k], 0)).sum(axis=0) + 1e-300)
    np.testing.assert_array_equal(part[:, 9:], 0.0)
    part2 = engine.breadth_partial(torch.from_numpy(c).cuda(), f).cpu().numpy()
    np.testing.assert_array_equal(part, part2)
