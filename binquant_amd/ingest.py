"""Wire-format kline ingest.

The reference decodes each websocket frame with json.loads
(producers/klines_connector.py:77-90), builds a KlineProduceModel of string
fields for closed candles (:148-164) and, downstream, the store coerces them
with pd.to_numeric (market_regime/market_state_store.py:82-83). Here a batch
of raw frames is parsed natively (bq_parse_kline_events, one pass, strtod =
the doubles Python's float() gives) into arrays, and closed candles go to the
device store in one launch (DeviceMarketStateStore.update_batch, timestamp =
close_time as in consumers/klines_provider.py:135-154).
"""

from __future__ import annotations

import ctypes
from collections.abc import Iterable
from dataclasses import dataclass

import numpy as np

from . import _lib

SYMBOL_BYTES = 32


@dataclass
class KlineBatch:
    symbols: list[str]
    open_time: np.ndarray    # int64 ms
    close_time: np.ndarray   # int64 ms
    open: np.ndarray
    high: np.ndarray
    low: np.ndarray
    close: np.ndarray
    volume: np.ndarray
    closed: np.ndarray       # bool ("x")
    n_bad: int

    def __len__(self) -> int:
        return len(self.symbols)

    def closed_only(self) -> "KlineBatch":
        m = self.closed
        return KlineBatch([s for s, k in zip(self.symbols, m) if k], self.open_time[m], self.close_time[m],
                          self.open[m], self.high[m], self.low[m], self.close[m], self.volume[m], self.closed[m],
                          self.n_bad)

    def produce_models(self) -> list[dict]:
        """KlineProduceModel-shaped dicts (string fields, klines_connector.py:153-164)."""
        return [
            dict(symbol=s, open_time=str(int(a)), close_time=str(int(b)), open_price=repr(float(o)),
                 high_price=repr(float(h)), low_price=repr(float(l)), close_price=repr(float(c)),
                 volume=repr(float(v)))
            for s, a, b, o, h, l, c, v in zip(self.symbols, self.open_time, self.close_time, self.open, self.high,
                                              self.low, self.close, self.volume)
        ]


def _join(frames: bytes | str | Iterable[bytes | str]) -> bytes:
    if isinstance(frames, bytes):
        return frames
    if isinstance(frames, str):
        return frames.encode()
    parts = [f.encode() if isinstance(f, str) else bytes(f) for f in frames]
    for p in parts:
        if b"\n" in p:
            raise ValueError("a frame may not contain a newline (frames are newline-separated)")
    return b"\n".join(parts)


def parse_kline_events(frames: bytes | str | Iterable[bytes | str]) -> KlineBatch:
    """Raw websocket frames (a list, or one newline-separated buffer) -> arrays."""
    buf = _join(frames)
    cap = buf.count(b"\n") + 1
    sym = np.zeros((cap, SYMBOL_BYTES), dtype=np.uint8)
    ot = np.empty(cap, dtype=np.int64)
    ct = np.empty(cap, dtype=np.int64)
    f = np.empty((5, cap), dtype=np.float64)
    closed = np.empty(cap, dtype=np.uint8)
    n = ctypes.c_int64()
    bad = ctypes.c_int64()
    st = _lib.load().bq_parse_kline_events(
        buf, len(buf), cap, ctypes.c_void_p(sym.ctypes.data), SYMBOL_BYTES, ctypes.c_void_p(ot.ctypes.data),
        ctypes.c_void_p(ct.ctypes.data), _lib.ptr_array([f[i].ctypes.data for i in range(5)]),
        ctypes.c_void_p(closed.ctypes.data), ctypes.byref(n), ctypes.byref(bad),
    )
    _lib.check(st, "bq_parse_kline_events")
    k = n.value
    names = [bytes(r[: np.argmax(r == 0) if (r == 0).any() else SYMBOL_BYTES]).decode() for r in sym[:k]]
    return KlineBatch(names, ot[:k].copy(), ct[:k].copy(), *(f[i, :k].copy() for i in range(5)),
                      closed[:k].astype(bool), bad.value)


def ingest_kline_events(store, frames) -> KlineBatch:
    """Parse a batch of frames and append the closed candles to a
    DeviceMarketStateStore in one device update. Returns the closed batch."""
    b = parse_kline_events(frames).closed_only()
    if len(b):
        store.update_batch(b.symbols, b.close_time, b.open, b.high, b.low, b.close, b.volume)
    return b
