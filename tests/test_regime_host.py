"""CPU: the product's vectorised context scoring + market-regime annotation
(binquant_amd.market_regime.regime) against the reference's golden contexts,
fed with partial sums reduced (in numpy) from the oracle's per-symbol features."""

import json
from pathlib import Path

import numpy as np
import pytest

from binquant_amd.market_regime.regime import annotate_market, annotate_symbols, score_contexts
from oracle import market_ref

G = Path(__file__).resolve().parent / "golden"
LABELS = ["trend_up_40", "random_64", "selloff_64"]


def partials_for(h, l, c, t, max_bars):
    rows = [market_ref.panel_features_at(h[i], l[i], c[i], t, max_bars) for i in range(c.shape[0])]
    P = np.zeros(10)
    for f in rows:
        if f is None:
            continue
        P += [1, f["return_pct"] > 0, f["return_pct"] < 0, f["above_ema20"], f["above_ema50"], f["return_pct"],
              f["trend_score"], f["atr_pct"], f["bb_width"], 0.0]
    return P, rows


@pytest.mark.parametrize("label", LABELS)
def test_vectorised_scoring_matches_reference(label):
    meta = json.loads((G / "market_context.json").read_text())
    panels = np.load(G / "market_context_panels.npz")
    sc = meta[label]
    ts_all = panels[f"{label}__timestamp"][0]
    h, l, c = (panels[f"{label}__{k}"] for k in ("high", "low", "close"))
    idx = [int(np.flatnonzero(ts_all == ts)[0]) for ts in sc["timestamps"]]
    btc_i = sc["symbols"].index(sc["btc"])
    parts, btc_ret, btc_trend, btc_ok, rows_at = [], [], [], [], []
    for t in idx:
        P, rows = partials_for(h, l, c, t, sc["max_bars"])
        parts.append(P)
        rows_at.append(rows)
        b = rows[btc_i]
        btc_ok.append(b is not None)
        btc_ret.append(b["return_pct"] if b else 0.0)
        btc_trend.append(b["trend_score"] if b else 0.0)
    batch = score_contexts(np.array(parts), np.array(btc_ret), np.array(btc_trend), np.array(btc_ok),
                           total_tracked=len(sc["symbols"]), timestamps=np.array(sc["timestamps"]))
    annotate_market(batch)
    for i, want in enumerate(sc["contexts"]):
        got = batch.context_at(i)
        if want is None:
            assert got is None
            continue
        assert got is not None
        for k, v in want.items():
            if k in ("symbol_features", "metadata", "btc_symbol", "confidence", "is_provisional", "timestamp"):
                continue
            if isinstance(v, bool) or v is None or isinstance(v, str) or isinstance(v, int):
                assert got[k] == v, (k, got[k], v)
            else:
                assert got[k] == pytest.approx(v, rel=1e-11, abs=1e-13), k
        # per-symbol micro regimes (element-wise annotation)
        rows = rows_at[i]
        syms = [s for s, r in zip(sc["symbols"], rows) if r is not None]
        rs = np.array([0.0 if s == sc["btc"] else r["return_pct"] - rows[btc_i]["return_pct"]
                       for s, r in zip(sc["symbols"], rows) if r is not None])
        valid_rows = [r for r in rows if r is not None]
        ann = annotate_symbols(
            [r["trend_score"] for r in valid_rows], [r["above_ema20"] for r in valid_rows],
            [r["above_ema50"] for r in valid_rows], rs, [r["bb_width"] for r in valid_rows],
            [r["atr_pct"] for r in valid_rows], [r["return_pct"] for r in valid_rows])
        for j, s in enumerate(syms):
            wf = want["symbol_features"][s]
            assert ann["micro_regime"][j] == wf["micro_regime"], s
            assert ann["micro_regime_strength"][j] == pytest.approx(wf["micro_regime_strength"], abs=1e-12)


@pytest.mark.parametrize("seed", range(6))
def test_vectorised_annotation_chain_matches_sequential(seed):
    """annotate_market over T timestamps at once (predecessor arrays, run
    starts by a running max) against the oracle's one-context-at-a-time
    _annotate_market_regime chained through each previous valid context
    (accumulator._get_previous_context): regimes, transitions, strengths and
    regime_stable_since equal on random partials with gaps in validity and
    every kind of seed context."""
    rng = np.random.default_rng(seed)
    T, S = 400, 120
    n = np.where(rng.random(T) < 0.15, rng.integers(0, 60, T), S).astype(float)
    adv = np.floor(n * rng.random(T))
    dec = np.floor((n - adv) * rng.random(T))
    P = np.stack([n, adv, dec, np.floor(n * rng.random(T)), np.floor(n * rng.random(T)),
                  rng.normal(0, 0.03, T) * n, rng.normal(0, 0.01, T) * n, rng.uniform(0, 0.06, T) * n,
                  rng.uniform(0, 0.25, T) * n, np.zeros(T)], 1)
    br, bt, bv = rng.normal(0, 0.03, T), rng.normal(0, 0.02, T), rng.random(T) > 0.1
    ts = 1_700_000_000_000 + 900_000 * np.arange(T)
    seeds = [None, {"market_regime": None},
             {"market_regime": "RANGE", "long_regime_score": 0.3, "short_regime_score": 0.2,
              "range_regime_score": 0.6, "stress_regime_score": 0.1, "regime_stable_since": 5},
             {"market_regime": "TRANSITIONAL", "long_regime_score": 0.3, "short_regime_score": 0.3,
              "range_regime_score": 0.3, "stress_regime_score": 0.3}]
    for seed_ctx in seeds:
        batch = annotate_market(score_contexts(P, br, bt, bv, total_tracked=S, timestamps=ts), seed_ctx)
        prev = seed_ctx
        for i in range(T):
            got = batch.context_at(i)
            if got is None:
                continue
            want = market_ref.annotate_market(got, prev)
            for k in ("market_regime", "previous_market_regime", "market_regime_transition",
                      "market_regime_transition_strength", "regime_is_transitioning", "regime_stable_since",
                      "long_regime_score", "short_regime_score", "range_regime_score", "stress_regime_score"):
                assert got[k] == want[k], (seed_ctx, i, k, got[k], want[k])
            prev = want
