"""Deterministic synthetic kline panels for the panel-size golden fixtures.

Shared by tests/golden/make_golden.py (which runs the REAL reference functions
on these inputs in this container) and the GPU tests (which regenerate the
same inputs on the box and compare the device pipelines with the recorded
reference outputs). Only numpy's default_rng is used, and the fixture stores
a digest of the generated inputs, so a generator drift shows up as a digest
mismatch rather than as a parity failure.

Panel content (SURVEY §8c edge cases): per-symbol seeds and price scales
10^U(-3, 4); halted stretches (open = high = low = close constant, zero
volume); isolated zero-volume bars; volume and price spikes (so the burst /
pump / spike detectors fire); a benchmark (BTC) series with missing candles.
"""

from __future__ import annotations

import hashlib

import numpy as np

FIELDS = ("open", "high", "low", "close", "volume", "quote_asset_volume")


def strategy_panel(S: int = 64, T: int = 1100, seed: int = 2026) -> dict[str, np.ndarray]:
    out = {f: np.empty((S, T)) for f in FIELDS}
    for s in range(S):
        g = np.random.default_rng(seed * 1000 + s)
        scale = 10.0 ** g.uniform(-3.0, 4.0)
        vol = g.uniform(0.002, 0.01)
        c = scale * np.exp(np.cumsum(g.normal(0.0, vol, T)))
        v = g.lognormal(3.0, 1.0, T)
        for j in g.choice(np.arange(30, T - 2), 14, replace=False):   # spikes
            v[j] *= g.uniform(3.0, 10.0)
            c[j] *= 1.0 + g.choice([-1.0, 1.0]) * g.uniform(0.01, 0.06)
        o = np.r_[c[0], c[:-1]]
        h = np.maximum(o, c) * (1.0 + g.uniform(0.0, 0.003, T))
        l = np.minimum(o, c) * (1.0 - g.uniform(0.0, 0.003, T))
        if s % 5 == 1:   # a halted stretch: flat bars, no volume
            a = int(g.integers(100, T - 80))
            c[a : a + 40] = c[a]
            o[a : a + 40] = h[a : a + 40] = l[a : a + 40] = c[a]
            v[a : a + 40] = 0.0
            o[a + 40] = c[a]
            h[a + 40] = max(h[a + 40], o[a + 40])
            l[a + 40] = min(l[a + 40], o[a + 40])
        zero = g.random(T) < 0.004
        v[zero] = 0.0
        out["open"][s], out["high"][s], out["low"][s], out["close"][s], out["volume"][s] = o, h, l, c, v
        out["quote_asset_volume"][s] = v * c
    return out


def btc_series(T: int = 1100, seed: int = 2026) -> tuple[np.ndarray, np.ndarray]:
    """(keep mask, close) of the benchmark: 60k-scale walk, ~2% of candles
    missing (runs of 1-3), so the left merge on open_time leaves NaN gaps."""
    g = np.random.default_rng(seed + 99)
    c = 60000.0 * np.exp(np.cumsum(g.normal(0.0, 0.004, T)))
    keep = np.ones(T, bool)
    for j in g.choice(np.arange(5, T - 5), 8, replace=False):
        keep[j : j + int(g.integers(1, 4))] = False
    return keep, c


def sample_positions(S: int, T: int, k: int = 48, seed: int = 7) -> np.ndarray:
    """[S, k] sorted candle indices per symbol at which outputs are recorded:
    the last two rows (what the strategies consume), the 1024-candle tile
    boundary and random interior positions."""
    fixed = [t for t in (0, 1, 1022, 1023, 1024, 1025, T - 2, T - 1) if 0 <= t < T]
    g = np.random.default_rng(seed)
    rows = []
    for _ in range(S):
        rest = np.setdiff1d(np.arange(T), fixed)
        rows.append(np.sort(np.r_[fixed, g.choice(rest, k - len(fixed), replace=False)]))
    return np.array(rows, dtype=np.int64)


def digest(panel: dict[str, np.ndarray]) -> str:
    h = hashlib.sha256()
    for f in sorted(panel):
        h.update(f.encode())
        h.update(np.ascontiguousarray(panel[f], dtype=np.float64).tobytes())
    return h.hexdigest()
