"""Synthetic kline panels (SURVEY.md §8d generator).

close = p0 * exp(cumsum(N(0, 0.002))), open = previous close,
high/low = max/min(open, close) * (1 +/- U(0, 0.003)), volume ~ LogNormal(3, 1),
quote_asset_volume = volume * close, timestamps 60 000 ms apart. The C2-style
panel adds a per-symbol price scale 10^U(-4, 4), constant runs of 30 bars on
~1% of bars and zero-volume bars on ~0.5% of bars.

``numpy_panel`` is deterministic (per-symbol seeds) and is what the parity
tests use; ``device_panel`` draws the same distributions directly in HBM with
torch's generator for the large benchmark shapes.
"""

from __future__ import annotations

import numpy as np

FIELDS = ("open", "high", "low", "close", "volume")


def numpy_symbol(T: int, seed: int, scale: float = 100.0, edges: bool = False) -> dict[str, np.ndarray]:
    rng = np.random.default_rng(seed)
    ret = rng.normal(0.0, 0.002, T)
    close = scale * np.exp(np.cumsum(ret))
    if edges and T > 40:
        n_runs = max(1, T // 100 // 30 + (1 if T >= 100 else 0))
        for _ in range(n_runs):
            start = int(rng.integers(1, max(2, T - 30)))
            close[start : start + 30] = close[start]
    open_ = np.empty(T)
    open_[0] = close[0]
    open_[1:] = close[:-1]
    hi_n = rng.uniform(0.0, 0.003, T)
    lo_n = rng.uniform(0.0, 0.003, T)
    high = np.maximum(open_, close) * (1.0 + hi_n)
    low = np.minimum(open_, close) * (1.0 - lo_n)
    volume = rng.lognormal(3.0, 1.0, T)
    if edges:
        flat = close == np.roll(close, 1)
        flat[0] = False
        # a constant run is a halted market: flat bar, no range
        open_[flat] = close[flat]
        high[flat] = close[flat]
        low[flat] = close[flat]
        zero = rng.random(T) < 0.005
        volume[zero] = 0.0
    return {"open": open_, "high": high, "low": low, "close": close, "volume": volume}


def numpy_panel(S: int, T: int, seed0: int = 0, edges: bool = True, scales: bool = True) -> dict[str, np.ndarray]:
    """[S, T] float64 panel, symbol s drawn from seed seed0 + s."""
    out = {f: np.empty((S, T)) for f in FIELDS}
    srng = np.random.default_rng(10_000 + seed0)
    for s in range(S):
        scale = 10.0 ** srng.uniform(-4.0, 4.0) if scales else 100.0
        sym = numpy_symbol(T, seed0 + s, scale=scale, edges=edges)
        for f in FIELDS:
            out[f][s] = sym[f]
    return out


def device_panel(S: int, T: int, device="cuda", seed: int = 0, chunk: int = 12_500):
    """Same distributions, generated in HBM (no per-symbol seeds; for benches).

    Symbols are drawn in blocks of `chunk` rows straight into the five [S, T]
    outputs, so the generation temporaries stay at a few block-sized arrays
    (the 100k x 10k headline panel is 40 GB of inputs; unchunked temporaries
    would add as much again)."""
    import torch

    g = torch.Generator(device=device)
    g.manual_seed(seed)
    f64 = dict(dtype=torch.float64, device=device)
    out = {f: torch.empty((S, T), **f64) for f in FIELDS}
    for lo in range(0, S, max(1, chunk)):
        hi = min(S, lo + max(1, chunk))
        n = hi - lo
        scale = torch.pow(10.0, torch.empty((n, 1), **f64).uniform_(-4.0, 4.0, generator=g))
        close = out["close"][lo:hi]
        torch.cumsum(torch.empty((n, T), **f64).normal_(0.0, 0.002, generator=g), dim=1, out=close)
        close.exp_().mul_(scale)
        open_ = out["open"][lo:hi]
        open_[:, 0] = close[:, 0]
        open_[:, 1:] = close[:, :-1]
        u = torch.empty((n, T), **f64)
        torch.mul(torch.maximum(open_, close), u.uniform_(0.0, 0.003, generator=g).add_(1.0), out=out["high"][lo:hi])
        torch.mul(torch.minimum(open_, close), u.uniform_(0.0, 0.003, generator=g).neg_().add_(1.0),
                  out=out["low"][lo:hi])
        torch.exp(u.normal_(3.0, 1.0, generator=g), out=out["volume"][lo:hi])
        del u
    return out
