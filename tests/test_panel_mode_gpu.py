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


def _near(a, b, rtol=1e-9):
    """|a - b| within rtol of the larger magnitude (a comparison at a near-tie)"""
    with np.errstate(invalid="ignore"):
        return np.abs(a - b) <= rtol * np.maximum(np.abs(a), np.abs(b))


def _cooldown(label, bars):
    """FailedSpikeFade.apply_cooldown (strategies/failed_spike_fade.py:495-520) per row"""
    kept = np.zeros_like(label)
    for s in range(label.shape[0]):
        last = None
        for t in np.flatnonzero(label[s]):
            if last is None or t - last > bars:
                kept[s, t] = True
                last = t
    return kept


def _flip_causes_pump(x, y):
    """every score_cross flip sits where pump_score is within 1e-9 of its
    threshold at t or t - 1 (in either mode)"""
    flip = x["score_cross"] != y["score_cross"]
    tie = np.zeros_like(flip)
    for m in (x, y):
        nt = _near(m["pump_score"], m["score_threshold"])
        tie |= nt
        tie[:, 1:] |= nt[:, :-1]
    return flip, tie


def _flip_causes_spike(x, y, p):
    """FailedSpikeFade's flags: the primary comparisons (volume ratio vs the
    calibrated cluster ratio, |pct change| vs the dynamic threshold, the
    cumulative sums and the volume derivative vs their constants) flip only at
    near-ties of their own operands; every derived flag flips only where one of
    its primaries did (the cluster flag over its window, the labels through
    the combination), and each mode's label is the cooldown of its label_pre."""
    import pandas as pd

    bad = {}
    def prim(m):
        vr, vc = m["volume_ratio"], m["volume_cluster_min_ratio"][:, None]
        pca, thr, pc = m["price_change_abs"], m["price_break_threshold_series"], m["price_change"]
        cp = np.stack([pd.Series(r).clip(lower=0).rolling(p.cumulative_price_window).sum().to_numpy() for r in pc])
        cn = np.stack([pd.Series(r).clip(upper=0).abs().rolling(p.cumulative_price_window).sum().to_numpy()
                       for r in pc])
        vd = vr - np.concatenate([np.full((vr.shape[0], p.accel_volume_deriv_window), np.nan),
                                  vr[:, :-p.accel_volume_deriv_window]], axis=1)
        return dict(cond=(vr, np.broadcast_to(vc, vr.shape)), cond8=(vr, np.broadcast_to(vc * 0.8, vr.shape)),
                    pbf=(pca, thr),
                    cum_pos=(cp, np.full_like(cp, p.cumulative_price_threshold)),
                    cum_neg=(cn, np.full_like(cn, p.cumulative_price_threshold)),
                    acc=(vd, np.full_like(vd, p.accel_volume_deriv_min)))
    px, py = prim(x), prim(y)
    tie = {}
    for k in px:
        a, b = px[k], py[k]
        with np.errstate(invalid="ignore"):
            fx, fy = a[0] >= a[1], b[0] >= b[1]
        t = _near(*a) | _near(*b)
        bad[k] = int(((fx != fy) & ~t).sum())   # a primary comparison flipped away from a near-tie
        tie[k] = (fx != fy)
    W = p.volume_cluster_window
    cl = np.zeros_like(tie["cond"])
    for d in range(-1, W):   # the cluster count's window, and the 'last' mode's look-ahead
        if d >= 0:
            cl[:, d:] |= tie["cond"][:, :tie["cond"].shape[1] - d]
        else:
            cl[:, :-1] |= tie["cond"][:, 1:]
    c8 = np.zeros_like(tie["cond8"])   # the cumulative flags' volume gate: a rolling max of cond8
    for d in range(max(p.cumulative_price_window, 1)):
        c8[:, d:] |= tie["cond8"][:, :tie["cond8"].shape[1] - d]
    causes = {
        "volume_cluster_flag": cl, "price_break_flag": tie["pbf"],
        "cumulative_price_break_flag": tie["cum_pos"] | c8, "cumulative_price_break_short_flag": tie["cum_neg"] | c8,
        "accel_spike_flag": tie["acc"], "accel_spike_short_flag": tie["acc"],
    }
    combo = cl | tie["pbf"]
    causes["label_pre"] = combo | tie["cum_pos"] | c8 | tie["acc"]
    causes["label_short_pre"] = combo | tie["cum_neg"] | c8 | tie["acc"]
    for k, cause in causes.items():
        bad[k] = int(((x[k] != y[k]) & ~cause).sum())
    for m, name in ((x, "panel"), (y, "exact")):   # the labels are the cooldown of label_pre in each mode
        for lab, pre in (("label", "label_pre"), ("label_short", "label_short_pre")):
            bad[f"{name}.{lab}=cooldown"] = int((m[lab] != _cooldown(m[pre], p.post_spike_cooldown_bars)).sum())
    return bad


def test_strategies_panel_mode_vs_exact(cuda):
    """pump score / failed spike in panel mode against their bit-exact replay
    (exact=True) on a 256 x 2500 panel with halts and spikes: floats at 1e-9
    of each row's magnitude; every flag that differs is explained — its own
    comparison sits at a near-tie (operands within 1e-9 of each other in
    either mode), or it derives from such a flag (cluster window, label
    combination, cooldown) — and every flag whose operands are exact in both
    modes (colours, streaks) is equal. The five std columns (formed in the
    base pass in panel mode, pandas' replayed online variance in exact mode)
    follow tests/spike_std.py's rule, the compression flag equal away from
    near-ties of its operands."""
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
        x = {k: v.cpu().numpy() for k, v in a.items()}
        y = {k: v.cpu().numpy() for k, v in b.items()}
        skip = {}
        if name == "spike":   # the panel stds (base pass) vs the replays: tests/spike_std.py's rule
            from tests import spike_std

            skip = spike_std.check(x, y, {"close": p["close"], "volume": p["volume"],
                                          "body_size_pct": y["body_size_pct"]})
            for k, m in skip.items():
                x[k] = np.where(m, y[k], x[k])
        for k in y:
            if y[k].dtype == bool:
                continue
            with np.errstate(all="ignore"):
                fin = np.where(np.isfinite(y[k]), np.abs(y[k]), np.nan)
                sc = np.nan_to_num(np.nanmax(fin, axis=-1, initial=0.0), nan=1.0)
            sc = np.where(sc > 0, sc, 1.0)
            sc = sc[..., None] if y[k].ndim == 2 else sc
            assert_close(x[k], y[k], f"{name}.{k}", rtol=1e-9, scale=np.broadcast_to(sc, y[k].shape))
        if name == "pump":
            flip, tie = _flip_causes_pump(x, y)
            assert not (flip & ~tie).any(), ("score_cross flips away from a near-tie", int((flip & ~tie).sum()))
        else:
            bad = _flip_causes_spike(x, y, strategies.SpikeParams())
            assert not any(bad.values()), bad
            for k in ("is_bullish", "upward", "downward", "early_proba_aug_flag"):
                np.testing.assert_array_equal(x[k], y[k], err_msg=k)
            s8, s20 = y["rolling_price_std_8"], y["rolling_price_std_20"]   # the compression flag: near-ties only
            near = _near(s8, 0.6 * s20)
            assert not ((x["vol_compression_flag"] != y["vol_compression_flag"]) & ~near).any()


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
