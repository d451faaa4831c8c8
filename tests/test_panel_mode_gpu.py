"""Panel mode of bq_rolling_batch (bq_panel.hip, bq_roll_job.panel = 1): the
time-parallel rolling sum / mean and ewm against pandas itself on panels with
missing values (gaps, leading NaN, a row all NaN), constant runs (pandas'
same-value rule: exact values), signed values (calc_mean's sign rule), every
window / shift / min_periods combination the strategy pipelines use plus
edges — at 1e-9, constant windows exactly; and the strategy pipelines in
panel mode against the bit-exact replays (exact=True)."""

import numpy as np
import pandas as pd
import pytest
import torch

from binquant_amd import engine
from tests.util import assert_close

pytestmark = pytest.mark.gpu


def _panel(S, T, seed, signed=False):
    rng = np.random.default_rng(seed)
    x = np.exp(np.cumsum(rng.normal(0, 0.01, (S, T)), axis=1)) * 10 ** rng.uniform(-3, 4, (S, 1))
    if signed:
        x = x - np.median(x, axis=1, keepdims=True)
    x[0, 300:330] = x[0, 300]            # a constant run
    x[1, 500:502] = np.nan               # a gap
    x[2, :90] = np.nan                   # a late listing
    x[3, ::97] = np.nan                  # scattered gaps
    x[4, 2040:2060] = np.nan if T > 2060 else x[4, 2040:2060]   # across the tile boundary
    x[5] = np.nan                        # all missing
    x[6, 1000:1400] = 3.25               # a long constant run (past the window)
    x[7, 700:760] = 0.0                  # zeros
    if T > 2100:                         # runs crossing the 2048-candle tile boundary (the run-start carry)
        x[8, 2030:2100] = x[8, 2030]
        x[9, 2030:2100] = 0.0
    if T > 4150:                         # ... and the second one
        x[10, 4080:4150] = x[10, 4080]
        x[11, 4080:4150] = 0.0
    return x


@pytest.mark.parametrize("T", [700, 2048, 2500, 4500])
@pytest.mark.parametrize("signed", [False, True])
def test_panel_sum_mean_vs_pandas(cuda, T, signed):
    x = _panel(40, T, seed=T + signed, signed=signed)
    d = torch.from_numpy(x).cuda()
    cases = [(w, mp, sh, st) for st in ("sum", "mean") for (w, mp, sh) in
             ((2, 2, 0), (3, 3, 0), (5, 5, 0), (10, 10, 0), (12, 12, 0), (20, 20, 1), (20, 1, 1), (96, 96, 32),
              (7, 0, 3), (1, 1, 0), (48, 20, 5))]
    specs = [engine.Roll(d, w, st, min_periods=mp, shift=sh) for (w, mp, sh, st) in cases]
    for i in range(0, len(specs), 16):
        got = engine.rolling_many(*specs[i:i + 16], exact=False)
        for (w, mp, sh, st), g in zip(cases[i:i + 16], got):
            g = g.cpu().numpy()
            for s in range(x.shape[0]):
                r = pd.Series(x[s]).shift(sh).rolling(w, min_periods=mp)
                want = (r.sum() if st == "sum" else r.mean()).to_numpy()
                scale = np.nanmax(np.abs(x[s])) * w if np.isfinite(x[s]).any() else 1.0
                assert_close(g[s], want, f"{st} w={w} mp={mp} sh={sh} row {s}", rtol=1e-9, scale=scale)
                # constant windows: pandas returns the value exactly (same-value rule)
                if s in (0, 6, 8, 9, 10, 11):
                    const = pd.Series(x[s]).shift(sh).rolling(w, min_periods=max(mp, 1)).apply(
                        lambda a: float(np.all(a[~np.isnan(a)] == a[~np.isnan(a)][-1])) if (~np.isnan(a)).any()
                        else 0.0, raw=True).to_numpy() > 0
                    np.testing.assert_array_equal(g[s][const], want[const], err_msg=f"{st} constant w={w} row {s}")


@pytest.mark.parametrize("T", [700, 2049, 4500])
def test_panel_ewm_vs_pandas(cuda, T):
    x = _panel(40, T, seed=T + 7)
    d = torch.from_numpy(x).cuda()
    cases = [(1 / 14, 14), (2 / 21, 0), (2 / 51, 0), (0.5, 3), (1.0, 0), (0.01, 100)]
    got = engine.rolling_many(*[engine.Ewm(d, alpha=a, min_periods=m) for a, m in cases], exact=False)
    exact = engine.rolling_many(*[engine.Ewm(d, alpha=a, min_periods=m) for a, m in cases])
    for (a, m), g, e in zip(cases, got, exact):
        g, e = g.cpu().numpy(), e.cpu().numpy()
        for s in range(x.shape[0]):
            want = pd.Series(x[s]).ewm(alpha=a, adjust=False, min_periods=m).mean().to_numpy()
            scale = np.nanmax(np.abs(x[s])) if np.isfinite(x[s]).any() else 1.0
            assert_close(g[s], want, f"ewm a={a:.4f} mp={m} row {s}", rtol=1e-9, scale=scale)
            np.testing.assert_array_equal(e[s], want)   # the replay stays pandas' bits
        # rows with a missing value run pandas' recursion itself from the first gap
        for s in (1, 2, 3):
            want = pd.Series(x[s]).ewm(alpha=a, adjust=False, min_periods=m).mean().to_numpy()
            first = int(np.argmax(np.isnan(x[s])))
            tile = first // 2048 * 2048
            np.testing.assert_array_equal(g[s][tile:], want[tile:], err_msg=f"serial ewm row {s}")


def test_panel_benchmark_row_in_batch(cuda):
    """a [1, T] benchmark series with gaps beside an [S, T] panel (the pump
    score's layout) in one panel-mode batch"""
    S, T = 30, 1500
    x = _panel(S, T, seed=3)
    b = x[9:10].copy()
    b[0, ::13] = np.nan
    d, bd = torch.from_numpy(x).cuda(), torch.from_numpy(b).cuda()
    got = engine.rolling_many(engine.Ewm(d, span=20), engine.Ewm(bd, span=50), engine.Roll(d, 20, "mean", shift=1),
                              exact=False)
    assert got[1].shape == (1, T)
    want = pd.Series(b[0]).ewm(span=50, adjust=False).mean().to_numpy()
    assert_close(got[1].cpu().numpy()[0], want, "bench ewm50", rtol=1e-9, scale=np.nanmax(np.abs(b)))


def test_strategies_panel_mode_vs_exact(cuda):
    """pump score / failed spike in panel mode against their bit-exact replay
    (exact=True) on a 256 x 2500 panel with halts and spikes: floats at 1e-9
    of each row's magnitude, flags equal away from near-ties of the values
    they threshold (counted: at most a handful per million)"""
    from binquant_amd import strategies
    from binquant_amd.synth import numpy_panel

    S, T = 256, 2500
    p = numpy_panel(S, T, seed0=99, edges=True)
    d = {k: torch.from_numpy(v).cuda() for k, v in p.items()}
    qv = d["volume"] * d["close"]
    btc = d["close"][0].clone()
    btc[::17] = float("nan")
    for name, fn in (("pump", lambda ex: strategies.pump_score_features(d["open"], d["high"], d["low"], d["close"],
                                                                        d["volume"], btc, exact=ex)),
                     ("spike", lambda ex: strategies.failed_spike_features(d["open"], d["high"], d["low"], d["close"],
                                                                           d["volume"], qv, exact=ex))):
        a, b = fn(False), fn(True)
        flips = 0
        for k in b:
            x, y = a[k].cpu().numpy(), b[k].cpu().numpy()
            if y.dtype == bool:
                flips += int((x != y).sum())
                continue
            with np.errstate(all="ignore"):
                fin = np.where(np.isfinite(y), np.abs(y), np.nan)
                sc = np.nan_to_num(np.nanmax(fin, axis=-1, initial=0.0), nan=1.0)
            sc = np.where(sc > 0, sc, 1.0)
            sc = sc[..., None] if y.ndim == 2 else sc
            assert_close(x, y, f"{name}.{k}", rtol=1e-9, scale=np.broadcast_to(sc, y.shape))
        assert flips <= S * T * 5e-6, (name, flips)



def test_packed_rank_within_rounding(cuda):
    """Panel-mode order statistics on the tile kernels sort packed keys (the
    union slot in the key's low bits): every quantile / median / max equals
    the exact kernel's within 2^-44 relative (an element that close to the
    true order statistic), NaN warm-up and gaps identical — including windows
    of values that differ only in their last mantissa bits."""
    S, T = 48, 1500
    x = _panel(S, T, seed=13)
    rng = np.random.default_rng(2)
    base = 1.0 + rng.integers(0, 4, (4, T)) * 2.0 ** -50   # near-ties in the low bits
    x[8:12] = base * 100.0
    d = torch.from_numpy(x).cuda()
    cases = [(48, "quantile", 0.8, 0, 1), (60, "quantile", 0.85, 20, 0), (80, "quantile", 0.92, 20, 1),
             (96, "quantile", 0.5, 96, 0), (40, "median", 0.5, 40, 2), (64, "max", 1.0, 64, 0)]
    specs = [engine.Roll(d, w, st, q=q, min_periods=mp, shift=sh) for (w, st, q, mp, sh) in cases]
    packed = engine.rolling_many(*specs, exact=False)
    exact = engine.rolling_many(*specs)
    for (w, st, q, mp, sh), a, b in zip(cases, packed, exact):
        a, b = a.cpu().numpy(), b.cpu().numpy()
        np.testing.assert_array_equal(np.isnan(a), np.isnan(b), err_msg=f"{st} w={w}")
        ok = np.isnan(b) | (np.abs(a - b) <= 2.0 ** -44 * np.abs(b))
        assert ok.all(), (st, w, int((~ok).sum()))
