"""The failed-spike panel path's five rolling std columns against pandas'
(or its bit-exact replay's) values, and their descendants.

Panel mode forms the stds inside the base pass (bq_spike_base_std: window sums
about a reference inside the window — the window's variance to rounding),
where pandas' roll_var runs an online add / remove recurrence over the whole
row that drifts where the std is small against the values (after a halted
stretch, on high-priced rows: ~1e-8 .. 1e-6 relative). The rule, per std
value: within `rtol` of pandas, or — where pandas drifted — within `rtol` of
the exactly computed window std (oracle.indicators_ref.exact_std, rational
arithmetic) with pandas the one further from it. The descendants (the three
z-scores, the 8 / 20 ratio, the compression flag) likewise: within `rtol` of
pandas, or within `rtol` of their formula on the kernel's means with the exact
window stds, pandas further from it (the flag: equal to the exact-std
comparison away from near-ties).
"""

from __future__ import annotations

import numpy as np

from oracle.indicators_ref import exact_std

EPS = 1e-6
# detect() std column -> (input series, window; None = the base window)
STD_COLS = {"price_std": ("close", None), "volume_std": ("volume", None), "rolling_price_std_8": ("close", 8),
            "rolling_price_std_20": ("close", 20), "body_size_pct_std_10": ("body_size_pct", 10)}
# descendant -> the std columns it reads
DESC = {"price_zscore": ("price_std",), "volume_zscore": ("volume_std",), "body_size_pct_z": ("body_size_pct_std_10",),
        "std_ratio_8_20": ("rolling_price_std_8", "rolling_price_std_20"),
        "vol_compression_flag": ("rolling_price_std_8", "rolling_price_std_20")}


def _t_of(positions, s, i):
    return int(positions[s, i]) if positions is not None else int(i)


def check(got: dict, want: dict, series: dict, base_window: int = 12, positions=None, rtol: float = 1e-9,
          atol_rel: float = 1e-11, max_frac: float = 0.01) -> dict[str, np.ndarray]:
    """got / want: {column: [S, N]} (N = T, or the K recorded positions of
    `positions` [S, K]); series: full [S, T] rows of close, volume and
    body_size_pct. Asserts the rule above for the std columns and the
    descendants' formula where a std drifted; returns {column: mask} of the
    positions the caller must not compare got against want (explained)."""
    skip = {}
    for col, (key, w) in STD_COLS.items():
        if col not in want:
            continue
        w = base_window if w is None else w
        g, v = np.asarray(got[col], dtype=np.float64), np.asarray(want[col], dtype=np.float64)
        assert g.shape == v.shape, col
        np.testing.assert_array_equal(np.isnan(g), np.isnan(v), err_msg=f"{col}: NaN pattern")
        with np.errstate(all="ignore"):
            fin = np.where(np.isfinite(v), np.abs(v), np.nan)
            sc = np.nan_to_num(np.nanmax(fin, axis=1, initial=0.0), nan=1.0)
        sc = np.where(sc > 0, sc, 1.0)[:, None]
        lim = rtol * np.abs(v) + atol_rel * sc
        bad = ~(np.abs(g - v) <= lim) & ~np.isnan(v)
        assert bad.sum() <= max(8, max_frac * bad.size), (col, int(bad.sum()), "deviations from pandas")
        x = np.asarray(series[key], dtype=np.float64)
        for s, i in np.argwhere(bad):
            t = _t_of(positions, s, i)
            ex = exact_std(x[s, t - w + 1 : t + 1])
            tol = rtol * abs(ex) + atol_rel * sc[s, 0]
            assert abs(g[s, i] - ex) <= tol, f"{col}[{s},{t}]: got {g[s, i]!r}, exact {ex!r}, pandas {v[s, i]!r}"
            assert abs(v[s, i] - ex) > abs(g[s, i] - ex), f"{col}[{s},{t}]: pandas {v[s, i]!r} is closer to {ex!r}"
        skip[col] = bad
    # descendants: where one deviates from pandas beyond the bar, its formula
    # on the kernel's means with the EXACT window stds must agree within the
    # bar and pandas must be the one further from it (flags: equal to the
    # exact-std comparison, or at a near-tie of its operands)
    def ex_std(col, s, t):
        key, w = STD_COLS[col]
        w = base_window if w is None else w
        return exact_std(np.asarray(series[key], dtype=np.float64)[s, t - w + 1 : t + 1])

    for col in DESC:
        if col not in want:
            continue
        g, v = np.asarray(got[col]), np.asarray(want[col])
        if col == "vol_compression_flag":
            bad = g.astype(bool) != v.astype(bool)
        else:
            g, v = g.astype(np.float64), v.astype(np.float64)
            np.testing.assert_array_equal(np.isnan(g), np.isnan(v), err_msg=f"{col}: NaN pattern")
            with np.errstate(all="ignore"):
                fin = np.where(np.isfinite(v), np.abs(v), np.nan)
                sc = np.nan_to_num(np.nanmax(fin, axis=1, initial=0.0), nan=1.0)
            sc = np.where(sc > 0, sc, 1.0)[:, None]
            bad = ~(np.abs(g - v) <= rtol * np.abs(v) + atol_rel * sc) & ~np.isnan(v)
        assert bad.sum() <= max(8, max_frac * bad.size), (col, int(bad.sum()), "deviations from pandas")
        for s, i in np.argwhere(bad):
            t = _t_of(positions, s, i)
            if col == "vol_compression_flag":
                a, b = ex_std("rolling_price_std_8", s, t), 0.6 * ex_std("rolling_price_std_20", s, t)
                near = abs(a - b) <= 1e-9 * max(abs(a), abs(b))
                assert near or bool(g[s, i]) == (a < b), (col, s, t)
                continue
            if col == "std_ratio_8_20":
                f = ex_std("rolling_price_std_8", s, t) / (ex_std("rolling_price_std_20", s, t) + EPS)
                base = 0.0
            else:
                key, ma, sd = {"price_zscore": ("close", "price_ma", "price_std"),
                               "volume_zscore": ("volume", "volume_ma", "volume_std"),
                               "body_size_pct_z": ("body_size_pct", "body_size_pct_ma_10", "body_size_pct_std_10")}[col]
                xv = float(series[key][s, t])
                e = ex_std(sd, s, t)
                f = (xv - float(got[ma][s, i])) / (e + EPS)
                base = abs(xv) / (e + EPS)
            tol = rtol * abs(f) + 1e-13 * base + atol_rel * float(sc[s, 0])
            assert abs(float(g[s, i]) - f) <= tol, (col, s, t, float(g[s, i]), f, float(v[s, i]))
            assert abs(float(v[s, i]) - f) >= abs(float(g[s, i]) - f) - tol, (col, s, t, "pandas closer")
        skip[col] = bad
    return skip
