"""Device MarketStateStore + live context accumulator vs the REAL reference
under a scripted feed (tests/golden/store_sequence.json, written by
tests/golden/make_golden.py from market_regime/market_state_store.py and
market_regime/live_market_context_accumulator.py): REST history syncs with
shuffled / duplicated / NaN / string rows, live ticks with skipped symbols,
late corrections and out-of-order candles, history cap 30.

Histories, last-closed timestamps, fresh sets and integer context fields are
compared exactly; float context fields and per-symbol features within the
fp64 tolerance (sums arrive in a fixed order instead of Python's set order);
regime / transition labels exactly."""

import json
from pathlib import Path

import numpy as np
import pandas as pd
import pytest
import torch

pytestmark = pytest.mark.gpu
G = Path(__file__).resolve().parent / "golden"

INT_KEYS = {"fresh_count", "total_tracked_symbols", "advancers", "decliners", "regime_stable_since", "timestamp"}
LABEL_KEYS = {"market_regime", "previous_market_regime", "market_regime_transition", "btc_symbol",
              "btc_present", "is_provisional", "regime_is_transitioning"}


def _num_close(g, w, name):
    assert abs(g - w) <= 1e-9 * abs(w) + 1e-12, f"{name}: {g!r} != {w!r}"


def compare_context(got, want, where):
    if want is None:
        assert got is None, f"{where}: expected no context"
        return
    assert got is not None, f"{where}: expected a context at {want['timestamp']}"
    for k, w in want.items():
        if k in ("metadata", "symbol_features"):
            continue
        assert k in got, f"{where}: missing field {k}"
        g = got[k]
        if k in INT_KEYS or k in LABEL_KEYS or w is None or isinstance(w, (str, bool)):
            assert g == w, f"{where}.{k}: {g!r} != {w!r}"
        else:
            _num_close(float(g), float(w), f"{where}.{k}")
    for k in ("btc_fresh", "btc_used_for_regime", "fresh_symbol_count"):
        assert got["metadata"][k] == want["metadata"][k], f"{where}.metadata.{k}"
    if "symbol_features" in want:
        gs, ws = got["symbol_features"], want["symbol_features"]
        assert sorted(gs) == sorted(ws), f"{where}: fresh symbol sets differ"
        for sym, wf in ws.items():
            gf = gs[sym]
            for k, w in wf.items():
                if k in ("symbol", "timestamp", "above_ema20", "above_ema50", "micro_regime",
                         "micro_regime_transition") or w is None or isinstance(w, (str, bool)):
                    assert gf[k] == w, f"{where}.{sym}.{k}: {gf[k]!r} != {w!r}"
                else:
                    _num_close(float(gf[k]), float(w), f"{where}.{sym}.{k}")


def test_store_and_contexts_follow_the_reference(cuda):
    from binquant_amd.market_regime.store import DeviceLiveMarketContextAccumulator, DeviceMarketStateStore

    d = json.loads((G / "store_sequence.json").read_text())
    store = DeviceMarketStateStore(max_bars_per_symbol=d["max_bars"], capacity=8)   # forces two regrowths
    acc = DeviceLiveMarketContextAccumulator(store, btc_symbol=d["btc"])
    ctxs = iter(d["contexts"])
    for i, op in enumerate(d["ops"]):
        rows = op.get("rows")
        payload = rows[0] if rows is not None and len(rows) == 1 else (pd.DataFrame(rows) if rows else None)
        if op["op"] == "update":
            store.update(op["symbol"], payload)
        elif op["op"] == "on_closed_candle":
            compare_context(acc.on_closed_candle(op["symbol"], payload), next(ctxs), f"op{i}")
        else:
            compare_context(acc.refresh_context_for_timestamp(op["ts"]), next(ctxs), f"op{i}")
    fin = d["final"]
    assert store.get_tracked_symbols() == fin["tracked"]
    for s, w in fin["last_closed"].items():
        assert store.get_last_closed_timestamp(s) == w, s
    for ts, w in fin["fresh"].items():
        assert sorted(store.get_fresh_symbols(int(ts))) == w, ts
    hist = store.get_all_histories()
    for s, w in fin["histories"].items():
        g = hist[s]
        assert list(g["timestamp"]) == w["timestamp"], s
        for c in ("open", "high", "low", "close", "volume"):
            np.testing.assert_array_equal(g[c].to_numpy(), np.asarray(w[c], dtype=np.float64), err_msg=f"{s}.{c}")
        single = store.get_symbol_history(s)
        assert list(single["timestamp"]) == w["timestamp"]
    latest = acc.get_latest_context()
    assert (latest["timestamp"] if latest else None) == fin["latest_context_ts"]


def test_store_merge_edge_cases(cuda):
    """Appends past the cap, a run longer than the cap, replacement of the
    newest and of an inner candle, an older-than-everything candle on a full
    ring (dropped by tail), against a pandas model of MarketStateStore.update."""
    from binquant_amd.market_regime.store import DeviceMarketStateStore, normalize_candles

    M = 7
    st = DeviceMarketStateStore(max_bars_per_symbol=M, capacity=2)
    model: dict[str, pd.DataFrame] = {}

    def ref_update(sym, rows):
        h = model.get(sym, pd.DataFrame())
        h = pd.concat([h, normalize_candles(pd.DataFrame(rows))], ignore_index=True)
        h = h.drop_duplicates(subset=["timestamp"], keep="last").sort_values("timestamp").tail(M)
        model[sym] = h.reset_index(drop=True)

    def row(t, c):
        return dict(timestamp=t, open=c, high=c + 1, low=c - 1, close=c, volume=t / 10)

    script = [
        ("X", [row(t, 100 + t) for t in range(1, 4)]),                 # plain appends
        ("X", [row(t, 200 + t) for t in range(4, 20)]),                # run longer than the cap
        ("X", [row(19, 5.0)]),                                          # replace newest
        ("X", [row(15, 6.0)]),                                          # replace inner
        ("X", [row(2, 7.0)]),                                           # older than the whole ring
        ("X", [row(16, 8.0), row(30, 9.0), row(17, 1.0), row(30, 2.0)]),   # mixed run, dup keeps last
        ("Y", [row(5, 1.0), row(3, 2.0), row(4, 3.0)]),                 # unordered first sync
        ("Y", [row(1, 4.0), row(2, 5.0)]),                              # prepend (inner merge)
        ("Z", [row(1, 1.0)]),
        ("X", [row(31, 1.5), row(32, 2.5)]),
    ]
    for sym, rows in script:
        st.update(sym, pd.DataFrame(rows))
        ref_update(sym, rows)
        for s2, want in model.items():
            got = st.get_symbol_history(s2)
            np.testing.assert_array_equal(got["timestamp"].to_numpy(), want["timestamp"].to_numpy().astype(np.int64))
            for c in ("open", "high", "low", "close", "volume"):
                np.testing.assert_array_equal(got[c].to_numpy(), want[c].to_numpy(np.float64))
            assert st.get_last_closed_timestamp(s2) == int(want["timestamp"].iloc[-1])


def test_store_features_bit_exact_vs_reference_features(cuda):
    """bq_store_features replays pandas' recurrences: equal to
    _compute_symbol_features (tests/golden/market_features.npz, written by the
    reference) bit for bit."""
    from binquant_amd.market_regime.store import DeviceMarketStateStore

    z = np.load(G / "market_features.npz")
    names = list(z["names"])
    cols = list(z["feature_columns"])
    st = DeviceMarketStateStore(max_bars_per_symbol=512, capacity=len(names))
    for nme in names:
        h, l, c = z[f"{nme}__high"], z[f"{nme}__low"], z[f"{nme}__close"]
        st.update_batch([nme] * len(c), np.arange(len(c)) * 60_000, c, h, l, c, np.ones(len(c)))
    feats, close = st.features(torch.arange(len(names), dtype=torch.int64))
    f = {k: v.cpu().numpy() for k, v in feats.items()}
    c = close.cpu().numpy()
    for i, nme in enumerate(names):
        want = dict(zip(cols, z[f"{nme}__features"]))
        if bool(z[f"{nme}__none"]):
            assert np.isnan(f["return_pct"][i]), nme
            continue
        assert c[i] == want["close"], nme
        for k in ("return_pct", "ema20", "ema50", "trend_score", "atr_pct", "bb_width"):
            assert f[k][i] == want[k], f"{nme}.{k}: {f[k][i]!r} != {want[k]!r}"
        assert bool(c[i] > f["ema20"][i]) == bool(want["above_ema20"])
