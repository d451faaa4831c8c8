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
    for k in ("btc_fresh", "btc_used_for_regime", "fresh_symbol_count") if "metadata" in want else ():
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


@pytest.mark.parametrize("fixture", ["store_sequence.json", "store_gaps.json"])
def test_store_and_contexts_follow_the_reference(cuda, fixture):
    """store_gaps.json: candles missing high and / or low (None, strings,
    NaN — kept by the store, which drops only a missing close): the features'
    skip-NaN true range and min_periods=1 ATR window over such histories."""
    from binquant_amd.market_regime.store import DeviceLiveMarketContextAccumulator, DeviceMarketStateStore

    d = json.loads((G / fixture).read_text())
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


def _frames_for(syms, k, rng, step=900_000, t0=1_760_000_400_000, x=True):
    from tests.test_ingest import frame

    out = []
    for s in syms:
        c = 10 ** rng.uniform(-2, 3)
        o = c * (1 + rng.normal(0, 0.002))
        out.append(frame(s, t0 + k * step, repr(o), repr(max(o, c) * 1.001), repr(min(o, c) * 0.999), repr(c),
                         f"{rng.lognormal(3, 1):.6f}", x=x))
    return out


def test_wire_ingest_matches_reference_store_update(cuda):
    """Raw websocket frames -> native parse -> one device update, equal to
    MarketStateStore.update of each KlineProduceModel's strings (close_time
    as the store timestamp, klines_provider.py:135-154)."""
    from binquant_amd.ingest import ingest_kline_events, parse_kline_events
    from binquant_amd.market_regime.store import DeviceMarketStateStore

    rng = np.random.default_rng(11)
    syms = [f"W{i:03d}USDT" for i in range(300)]
    a = DeviceMarketStateStore(max_bars_per_symbol=16, capacity=64)
    b = DeviceMarketStateStore(max_bars_per_symbol=16, capacity=64)
    for k in range(20):
        frames = _frames_for(syms, k, rng, x=(k % 7 != 3))
        ingest_kline_events(a, frames)
        for m in parse_kline_events(frames).closed_only().produce_models():
            b.update(m["symbol"], dict(timestamp=m["close_time"], open=m["open_price"], high=m["high_price"],
                                       low=m["low_price"], close=m["close_price"], volume=m["volume"]))
    ha, hb = a.get_all_histories(), b.get_all_histories()
    assert sorted(ha) == sorted(hb) == syms
    for s in syms:
        pd.testing.assert_frame_equal(ha[s], hb[s])


def _sharded_worker(rank, world, port, q):
    import os

    import torch.distributed as dist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        q.put((rank, _run_ticks(rank, world)))
    finally:
        dist.destroy_process_group()


def _run_ticks(rank, world):
    from binquant_amd.market_regime.batch import shard_bounds
    from binquant_amd.market_regime.store import DeviceLiveMarketContextAccumulator, DeviceMarketStateStore

    syms = ["BTCUSDT"] + [f"S{i:02d}USDT" for i in range(1, 90)]
    lo, hi = shard_bounds(len(syms) - 1, world, rank)
    mine = ["BTCUSDT"] + syms[1 + lo : 1 + hi]   # the benchmark is replicated
    store = DeviceMarketStateStore(max_bars_per_symbol=40, capacity=16)
    acc = DeviceLiveMarketContextAccumulator(store, "BTCUSDT")
    out = []
    for k in range(30):
        rng = np.random.default_rng(k)
        c = 100 * np.exp(rng.normal(0.001, 0.01, len(syms)).cumsum() / 10)
        skip = rng.random(len(syms)) < 0.1
        skip[0] = k % 11 == 5   # BTC occasionally stale
        idx = [i for i, s in enumerate(syms) if s in mine and not skip[i]]
        ts = np.full(len(idx), 1_000 + 900_000 * k)
        cc = c[idx]
        ctx = acc.on_closed_candles([syms[i] for i in idx], ts, cc, cc * 1.002, cc * 0.997, cc, np.ones(len(idx)),
                                    at=1_000 + 900_000 * k)
        out.append(None if ctx is None else {kk: v for kk, v in ctx.items() if kk not in ("symbol_features", "metadata")})
    return out


def test_sharded_accumulator_matches_single_rank(cuda):
    """Symbols sharded over 2 ranks (BTC replicated), one all-reduce per
    context (gloo here; RCCL on a node): the same contexts as one rank."""
    import torch.multiprocessing as mp

    single = _run_ticks(0, 1)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 29500 + int(np.random.default_rng().integers(0, 2000))
    procs = [ctx.Process(target=_sharded_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=240) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert sum(c is not None for c in single) > 10
    for r in range(2):
        for i, (a, b) in enumerate(zip(res[r], single)):
            compare_context(a, b, f"rank{r}.tick{i}")


def test_batch_fast_path_equals_generic_update(cuda):
    """update_batch over a repeated, registration-ordered symbol list (one
    candle per slot: the sorts and the dedupe are skipped) leaves the same
    rings as the generic sort / dedupe path, with NaN closes dropped and an
    all-NaN tick ignored."""
    from binquant_amd.market_regime.store import DeviceMarketStateStore

    syms = [f"S{i:03d}USDT" for i in range(150)]
    fast = DeviceMarketStateStore(max_bars_per_symbol=16, capacity=64)
    slow = DeviceMarketStateStore(max_bars_per_symbol=16, capacity=64)
    for s in syms:
        fast._slot(s)
        slow._slot(s)
    rng = np.random.default_rng(7)
    for k in range(24):
        c = 100 * np.exp(rng.normal(0, 0.01, len(syms)))
        if k % 5 == 2:
            c[rng.random(len(syms)) < 0.2] = np.nan
        if k == 9:
            c[:] = np.nan
        ts = np.full(len(syms), 900_000 * k)
        fast.update_batch(syms, ts, c, c * 1.01, c * 0.99, c, np.full(len(syms), float(k)))
        assert fast._slot_cache[2]
        # the generic path: same candles, presented in reverse order
        r = slice(None, None, -1)
        slow.update_batch(syms[r], ts[r], c[r], (c * 1.01)[r], (c * 0.99)[r], c[r], np.full(len(syms), float(k)))
        assert not slow._slot_cache[2]
    a, b = fast.get_all_histories(), slow.get_all_histories()
    assert set(a) == set(b) == set(syms)
    for s in syms:
        pd.testing.assert_frame_equal(a[s], b[s], check_exact=True)
        assert len(a[s]) == 16
