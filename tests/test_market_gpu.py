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


def test_c5_features_and_breadth_at_shard_size(cuda):
    """BASELINE configs[4] (C5) per-GPU leg: bq_market_features +
    bq_breadth_partial over the 12 500 x 10 000 C4 shard under the 400-bar
    store cap. At sampled timestamps (warm-up rows, t < max_bars, the cap
    boundary, the last t) every symbol's features are checked against the
    oracle restatement of _compute_symbol_features
    (live_market_context_accumulator.py:244-297, vectorised over symbols and
    pinned bit-exact to the per-symbol form in tests/test_oracle_golden.py),
    the partial counts exactly and the sums at 1e-9; 64 symbols also go
    through the per-symbol oracle. Then host scoring of the partials equals
    scoring of the oracle's partials (_build_context :96-242)."""
    from binquant_amd.market_regime.batch import reduce_partials
    from binquant_amd.synth import device_panel

    S, T, M = 12_500, 10_000, 400
    p = device_panel(S, T, seed=5150)
    h, l, c = p["high"], p["low"], p["close"]
    del p
    f = engine.market_features(h, l, c, max_bars=M)
    part = engine.breadth_partial(c, f)
    part, n_total = reduce_partials(part, S)
    torch.cuda.synchronize()
    assert n_total == S
    part = part.cpu().numpy()
    sample_syms = np.unique(np.r_[0, S - 1, np.linspace(0, S - 1, 62).astype(int)])
    for t in (0, 1, 13, 19, 20, 398, 399, 400, 401, 5_000, 9_998, 9_999):
        s0 = max(0, t - M + 1)
        hw, lw, cw = (x[:, s0 : t + 1].cpu().numpy() for x in (h, l, c))
        got = {k: v[:, t].cpu().numpy() for k, v in f.items()}
        want = market_ref.window_features(hw, lw, cw)
        if want is None:   # a one-candle history: no features, nothing counted
            assert all(np.isnan(v).all() for v in got.values()), t
            np.testing.assert_array_equal(part[t, :9], 0.0)
            continue
        # price-valued columns scale with the close, the ratios are dimensionless
        # (the scales of test_features_match_reference_restatement)
        for k in FEATURE_COLUMNS:
            scale = np.abs(cw[:, -1]) if k in ("ema20", "ema50") else 1e-3
            assert_close(got[k], want[k], f"{k}@{t}", rtol=1e-9, scale=scale)
        close_t = cw[:, -1]
        for e in ("ema20", "ema50"):   # no close within tolerance of its EMA: counts are exact
            assert not (np.abs(close_t - want[e]) <= 1e-9 * np.abs(close_t)).any(), (t, e)
        wp = market_ref.partials_from_features(want)
        np.testing.assert_array_equal(part[t, :5], wp[:5], err_msg=f"counts@{t}")
        assert part[t, 9] == S
        for i in (5, 6, 7, 8):
            mag = {5: np.abs(want["return_pct"]), 6: np.abs(want["trend_score"]), 7: np.abs(want["atr_pct"]),
                   8: np.abs(want["bb_width"])}[i].sum()
            assert abs(part[t, i] - wp[i]) <= 1e-9 * mag + 1e-300, (t, i, part[t, i], wp[i])
        for s in sample_syms[:: 4 if t < 9_998 else 1]:
            one = market_ref.symbol_features(hw[s], lw[s], cw[s])
            for k in FEATURE_COLUMNS:
                sc = abs(one["close"]) if k in ("ema20", "ema50") else 1e-3
                assert_close([got[k][s]], [one[k]], f"{k}[{s}]@{t}", rtol=1e-9, scale=[sc])
        # host scoring of the device partials == scoring of the oracle partials
        bf = market_ref.symbol_features(hw[0], lw[0], cw[0])
        wp[9] = S
        ctxs = []
        for P in (part[t : t + 1], wp[None]):
            b = score_contexts(P, np.array([bf["return_pct"]]), np.array([bf["trend_score"]]), np.array([True]),
                               total_tracked=S, timestamps=np.array([t]))
            annotate_market(b)
            ctxs.append(b.context_at(0))
        dev_ctx, ctx = ctxs
        assert (dev_ctx is None) == (ctx is None)
        if ctx is not None:
            for k, v in ctx.items():
                if isinstance(v, (bool, str, int)) or v is None:
                    assert dev_ctx[k] == v, (t, k)
                elif isinstance(v, float):
                    assert dev_ctx[k] == pytest.approx(v, rel=1e-9, abs=1e-12), (t, k)


_IMPL_CHILD = """
import sys, numpy as np, torch
from binquant_amd import engine
from binquant_amd.synth import numpy_panel
out = {}
for S, T, M in ((7, 1300, 400), (5, 900, 200), (3, 600, 15), (4, 2049, 512)):
    p = numpy_panel(S, T, seed0=S * T + M)
    d = {k: torch.from_numpy(v).cuda() for k, v in p.items()}
    f = engine.market_features(d["high"], d["low"], d["close"], max_bars=M)
    for k, v in f.items():
        out[f"{S}_{T}_{M}_{k}"] = v.cpu().numpy()
# the reference's golden histories (market_features.npz), one row each
z = np.load(sys.argv[2])
for name in z["names"]:
    name = str(name)
    h, l, c = (torch.from_numpy(np.ascontiguousarray(z[f"{name}__{k}"]))[None].cuda() for k in ("high", "low", "close"))
    f = engine.market_features(h, l, c, max_bars=400)
    for k, v in f.items():
        out[f"golden_{name}_{k}"] = v[:, -1:].cpu().numpy()
np.savez(sys.argv[1], **out)
"""


def test_features_wave_and_block_kernels_agree(cuda, tmp_path):
    """bq_market_features' two kernels — one wave per symbol (the context
    kernel's feature pass, default) and one workgroup per symbol
    (BQ_MARKET_FEATURES_IMPL=block) — on the same panels: NaN positions equal,
    values within 1e-12 of each row's magnitude (their window sums and EMA
    history terms are associated differently); both against the reference's
    golden histories (market_features.npz; the panel wave kernel is otherwise
    never run at S = 1). The panel kernels take finite high / low / close
    (include/binquant_amd.h bq_market_features): a missing close never reaches
    _compute_symbol_features (MarketStateStore drops the candle,
    market_state_store.py:84), and candles missing high / low — which the
    store keeps — go through the device store's pandas replay
    (tests/test_store_gpu.py, store_gaps.json)."""
    import os
    import subprocess
    import sys
    from pathlib import Path

    root = str(Path(__file__).resolve().parent.parent)
    res = {}
    for impl in ("wave", "block"):
        out = tmp_path / f"{impl}.npz"
        env = dict(os.environ, BQ_MARKET_FEATURES_IMPL=impl, PYTHONPATH=root)
        subprocess.run([sys.executable, "-c", _IMPL_CHILD, str(out), str(G / "market_features.npz")], env=env,
                       check=True, timeout=240)
        res[impl] = np.load(out)
    a, b = res["wave"], res["block"]
    assert set(a.files) == set(b.files)
    z = np.load(G / "market_features.npz")
    cols = [str(c) for c in z["feature_columns"]]
    for r in (a, b):   # the golden histories through each kernel
        for name in z["names"]:
            name = str(name)
            got = {k: float(r[f"golden_{name}_{k}"][0, 0]) for k in FEATURE_COLUMNS}
            if bool(z[f"{name}__none"]):
                assert all(np.isnan(v) for v in got.values()), name
                continue
            want = dict(zip(cols, z[f"{name}__features"]))
            for k in FEATURE_COLUMNS:
                assert_close([got[k]], [want[k]], f"{name}.{k}", scale=[abs(want["close"]) * 1e-2 + 1e-300])
    for k in a.files:
        x, y = a[k], b[k]
        np.testing.assert_array_equal(np.isnan(x), np.isnan(y), err_msg=k)
        fin = ~np.isnan(y)
        sc = np.nanmax(np.abs(np.where(fin, y, np.nan)), axis=1, keepdims=True)
        sc = np.where(np.isfinite(sc) & (sc > 0), sc, 1.0)
        assert np.all(np.abs(x - y)[fin] <= (1e-12 * np.broadcast_to(sc, y.shape))[fin]), k
