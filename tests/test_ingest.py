"""CPU tests of the native websocket-frame parser (bq_parse_kline_events,
host code in the C-ABI library) against the reference's own decode path:
json.loads of each frame (producers/klines_connector.py:77-90), "kline"
events only, fields s/t/T/o/h/l/c/v/x (:148-164), numbers coerced like
float() / pd.to_numeric (market_state_store.py:82-83) — bit-exact."""

import json

import numpy as np
import pytest

from binquant_amd.ingest import parse_kline_events


def frame(sym, t, o, h, l, c, v, x=True, extra=True, order=None):
    k = {"t": t, "T": t + 899_999, "s": sym, "i": "15m", "f": 1, "L": 2, "o": o, "c": c, "h": h, "l": l, "v": v,
         "n": 12, "x": x, "q": "1.5", "V": "0.5", "Q": "0.25", "B": "0"}
    if order is not None:
        k = {kk: k[kk] for kk in order}
    ev = {"e": "kline", "E": t + 5, "s": sym, "k": k}
    if extra:
        ev["z"] = {"nested": [1, {"a": "}"}, "x\"y"]}
    return json.dumps(ev)


def reference_decode(frames):
    rows = []
    for raw in frames:
        try:
            res = json.loads(raw)
        except Exception:
            continue
        if res.get("e") != "kline":
            continue
        k = res["k"]
        rows.append((k["s"], int(k["t"]), int(k["T"]), float(k["o"]), float(k["h"]), float(k["l"]),
                     float(k["c"]), float(k["v"]), bool(k["x"])))
    return rows


def random_frames(n, seed=0):
    rng = np.random.default_rng(seed)
    out = []
    for i in range(n):
        p = 10 ** rng.uniform(-8, 5)
        vals = [repr(float(p * (1 + rng.normal(0, 0.01)))) for _ in range(4)]
        vals = [f"{float(v):.{int(rng.integers(1, 18))}g}" if rng.random() < 0.5 else v for v in vals]
        vol = f"{rng.lognormal(3, 2):.8f}"
        out.append(frame(f"SYM{i % 37}USDT", 1_700_000_000_000 + 900_000 * i, *vals, vol, x=bool(rng.random() < 0.8),
                         extra=bool(i % 2)))
    return out


def test_parser_matches_json_loads_and_float():
    frames = random_frames(500)
    got = parse_kline_events(frames)
    want = reference_decode(frames)
    assert len(got) == len(want) and got.n_bad == 0
    for i, w in enumerate(want):
        assert got.symbols[i] == w[0]
        assert got.open_time[i] == w[1] and got.close_time[i] == w[2]
        for arr, x in zip((got.open, got.high, got.low, got.close, got.volume), w[3:8]):
            assert arr[i] == x   # bit-exact: strtod and float() both round correctly
        assert bool(got.closed[i]) == w[8]


def test_non_kline_and_malformed_frames():
    good = frame("AAAUSDT", 1, "1.5", "2", "1", "1.75", "10")
    frames = [
        good,
        json.dumps({"e": "24hrTicker", "s": "AAAUSDT", "k": {"junk": 1}}),   # not a kline: skipped
        json.dumps({"result": None, "id": 1}),                                 # subscription ack: skipped
        frame("BBBUSDT", 2, "abc", "2", "1", "1", "1"),                        # malformed number: bad
        json.dumps({"e": "kline", "k": {"t": 1, "s": "CCC"}}),                 # missing fields: bad
        "   ",                                                                  # blank line: ignored
        frame("DDDUSDT", 3, 4, 5, 3, 4.5, 9, order=["x", "v", "l", "h", "c", "o", "s", "T", "t"]),  # numbers, reordered
    ]
    got = parse_kline_events(frames)
    assert got.symbols == ["AAAUSDT", "DDDUSDT"] and got.n_bad == 2
    assert got.close.tolist() == [1.75, 4.5] and got.closed.tolist() == [True, True]


def test_closed_only_and_produce_models():
    frames = random_frames(50, seed=3)
    b = parse_kline_events(frames)
    c = b.closed_only()
    assert len(c) == int(b.closed.sum()) and c.closed.all()
    models = c.produce_models()
    assert set(models[0]) == {"symbol", "open_time", "close_time", "open_price", "high_price", "low_price",
                              "close_price", "volume"}
    assert float(models[0]["close_price"]) == c.close[0]


def test_single_buffer_and_newline_guard():
    frames = random_frames(10, seed=5)
    a = parse_kline_events(frames)
    b = parse_kline_events("\n".join(frames).encode())
    assert a.symbols == b.symbols and (a.close == b.close).all()
    with pytest.raises(ValueError):
        parse_kline_events(["{}\n{}"])
