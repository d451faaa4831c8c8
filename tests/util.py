"""Shared assertions for parity tests (tolerances stated here, used everywhere)."""

from __future__ import annotations

import numpy as np

# fp64 relative tolerance vs pandas for SMA/BB/ATR/EMA/RSI/MFI over <= 10k bars
# (SURVEY.md §8c): 1e-9 relative, plus an absolute floor scaled to the series
# magnitude for values that are near zero by cancellation (macd, std near 0).
RTOL = 1e-9
ATOL_REL = 1e-11


def assert_close(got, want, name: str, rtol: float = RTOL, scale=None, atol_rel: float = ATOL_REL):
    got = np.asarray(got, dtype=np.float64)
    want = np.asarray(want, dtype=np.float64)
    assert got.shape == want.shape, f"{name}: shape {got.shape} != {want.shape}"
    gn, wn = np.isnan(got), np.isnan(want)
    bad_nan = gn != wn
    assert not bad_nan.any(), (
        f"{name}: NaN mismatch at {np.argwhere(bad_nan)[:5].tolist()} "
        f"(got {got[bad_nan][:5]}, want {want[bad_nan][:5]})"
    )
    m = ~wn
    if not m.any():
        return
    g, w = got[m], want[m]
    inf_g, inf_w = np.isinf(g), np.isinf(w)
    assert (inf_g == inf_w).all() and (g[inf_g] == w[inf_w]).all(), f"{name}: inf mismatch"
    fin = ~inf_w
    g, w = g[fin], w[fin]
    if scale is None:
        atol = atol_rel * (np.max(np.abs(w)) if w.size else 0.0)
    else:
        s = np.broadcast_to(np.asarray(scale, dtype=np.float64), got.shape)[m][fin]
        atol = atol_rel * s
    err = np.abs(g - w)
    lim = rtol * np.abs(w) + atol
    if not (err <= lim).all():
        i = int(np.argmax(err - lim))
        raise AssertionError(
            f"{name}: max violation got={g[i]!r} want={w[i]!r} err={err[i]:.3e} lim={np.ravel(lim)[i] if np.ndim(lim) else lim:.3e} "
            f"({int((err > lim).sum())} of {err.size} elements)"
        )


def assert_close_or_exact(got, want, x, window: int, exact_fn, name: str, rtol: float = RTOL, scale=1.0,
                          max_cases: int | None = None):
    """assert_close, except where got and pandas' value differ beyond the
    tolerance: there got must equal the exactly computed value
    exact_fn(x[row, t - window + 1 : t + 1]) within rtol and pandas must be the
    one further from it (pandas' online rolling variance drifts in nearly
    constant windows; the kernels compute those windows exactly)."""
    got = np.asarray(got, dtype=np.float64)
    want = np.asarray(want, dtype=np.float64)
    x = np.asarray(x, dtype=np.float64)
    if got.ndim == 1:
        got, want, x = got[None], want[None], x[None]
    sc = np.broadcast_to(np.asarray(scale, dtype=np.float64), got.shape)
    bad = ~(np.abs(got - want) <= rtol * np.abs(want) + ATOL_REL * sc) & ~(np.isnan(got) & np.isnan(want))
    if max_cases is not None:
        assert bad.sum() <= max_cases, f"{name}: {int(bad.sum())} deviations from pandas"
    for s, t in np.argwhere(bad):
        ex = exact_fn(x[s, t - window + 1 : t + 1])
        tol = rtol * max(abs(ex), 1.0)
        assert abs(got[s, t] - ex) <= tol, f"{name}[{s},{t}]: got {got[s, t]!r}, exact {ex!r}, pandas {want[s, t]!r}"
        assert abs(want[s, t] - ex) > abs(got[s, t] - ex), f"{name}[{s},{t}]: pandas {want[s, t]!r} is closer to {ex!r}"
