"""GPU parity: the fused bq_enrich kernel vs the pandas oracle (per-symbol
reference call pattern of producers/context_evaluator.py:240-263).

Tolerances (tests/util.py): fp64 rtol 1e-9 + atol 1e-11 x series magnitude.
Derived threshold signals are compared exactly away from the tolerance band.
"""

import numpy as np
import pandas as pd
import pytest
import torch

from binquant_amd import engine
from binquant_amd.synth import numpy_panel
from oracle import indicators_ref as ref
from tests.util import assert_close

pytestmark = pytest.mark.gpu

COLS = ref.CANONICAL


def run_gpu(panel, params=None, columns=COLS, dev="cuda"):
    t = {k: torch.from_numpy(np.ascontiguousarray(v)).to(dev) for k, v in panel.items()}
    out = engine.enrich(t["open"], t["high"], t["low"], t["close"], t["volume"], params=params, columns=columns)
    torch.cuda.synchronize()
    return {k: v.cpu().numpy() for k, v in out.items()}


def compare(got, want, panel, cols=COLS):
    price = np.abs(panel["close"]).mean(axis=1, keepdims=True)
    for k in cols:
        if k in ("rsi", "mfi"):
            scale = 100.0
        elif k in ("macd", "macd_signal"):
            scale = price
        else:
            scale = price
        assert_close(got[k], want[k], k, scale=scale)


@pytest.mark.parametrize("S,T", [(64, 1000), (16, 3100), (8, 1024), (8, 1025), (4, 2048)])
def test_enrich_matches_oracle(cuda, S, T):
    panel = numpy_panel(S, T, seed0=S * 7 + T)
    got = run_gpu(panel)
    want = ref.enrich_panel(panel["open"], panel["high"], panel["low"], panel["close"], panel["volume"])
    compare(got, want, panel)


@pytest.mark.parametrize("T", [1, 2, 3, 7, 13, 14, 20, 99, 100, 101, 127, 128, 129, 1023])
def test_enrich_short_and_boundary_lengths(cuda, T):
    panel = numpy_panel(3, T, seed0=T, edges=False)
    got = run_gpu(panel)
    want = ref.enrich_panel(panel["open"], panel["high"], panel["low"], panel["close"], panel["volume"])
    compare(got, want, panel)


def test_constant_windows_are_exact(cuda):
    """pandas returns the value itself / std 0 on constant windows
    (SURVEY §7 hard parts): [0.3]*n must give ma == 0.3 exactly, std == 0."""
    T = 2500
    c = np.full(T, 0.3)
    c[:50] = np.linspace(0.2, 0.4, 50)
    c[1500:1600] = 7.1
    c[1600:] = 7.1 + np.cumsum(np.full(T - 1600, 1e-3))
    panel = {"open": c.copy(), "high": c * 1.0, "low": c * 1.0, "close": c, "volume": np.full(T, 5.0)}
    panel = {k: v[None, :].copy() for k, v in panel.items()}
    got = run_gpu(panel)
    want = ref.enrich_panel(panel["open"], panel["high"], panel["low"], panel["close"], panel["volume"])
    for k in ("ma_7", "ma_25", "ma_100", "bb_mid", "bb_upper", "bb_lower", "twap", "ATR"):
        m = ~np.isnan(want[k])
        np.testing.assert_array_equal(got[k][m][200:1400], want[k][m][200:1400], err_msg=k)
    assert (got["bb_upper"][0, 1550:1600] == 7.1).all()
    compare(got, want, panel)


def test_zero_volume_and_flat_bars(cuda):
    panel = numpy_panel(4, 1500, seed0=99, edges=True)
    panel["volume"][:, 100:130] = 0.0
    got = run_gpu(panel)
    want = ref.enrich_panel(panel["open"], panel["high"], panel["low"], panel["close"], panel["volume"])
    compare(got, want, panel)


def test_subset_of_columns_and_params(cuda):
    panel = numpy_panel(8, 700, seed0=5)
    p = engine.IndicatorParams(ma_periods=(5, 30, 126), rsi_window=9, bb_window=10, bb_ddof=0, bb_k=2.5,
                               atr_window=21, twap_window=8, ema_spans=(9, 34), mfi_window=10,
                               macd_fast=8, macd_slow=21, macd_signal=5)
    cols = ("ma_7", "ma_100", "rsi", "bb_upper", "bb_lower", "ATR", "mfi", "macd_signal", "ema50")
    got = run_gpu(panel, params=p, columns=cols)
    rename = {"ma_7": "ma_5", "ma_100": "ma_126", "ema50": "ema34"}
    # oracle names columns by period; map the canonical slot names
    want_cols = {}
    for s in range(8):
        df = pd.DataFrame({k: panel[k][s] for k in panel})
        df = ref.indicators_enrichment(df, p.as_oracle_dict())
        for k in cols:
            want_cols.setdefault(k, []).append(df[rename.get(k, k)].to_numpy())
    want = {k: np.stack(v) for k, v in want_cols.items()}
    compare(got, want, panel, cols)


def test_derived_signals_exact_away_from_boundary(cuda):
    """Crossovers / thresholds agree exactly except within tolerance of the cut."""
    panel = numpy_panel(32, 1200, seed0=3)
    got = run_gpu(panel)
    want = ref.enrich_panel(panel["open"], panel["high"], panel["low"], panel["close"], panel["volume"])
    c = panel["close"]
    tol = 1e-9 * np.abs(c)
    for a, b in (("ema20", None), ("ema50", None), ("bb_upper", None), ("bb_lower", None), ("ma_25", None)):
        w, g = want[a], got[a]
        m = ~np.isnan(w) & (np.abs(c - w) > 10 * tol)
        np.testing.assert_array_equal((c > g)[m], (c > w)[m], err_msg=a)
    for k, cut in (("rsi", 30.0), ("rsi", 70.0), ("mfi", 50.0)):
        w, g = want[k], got[k]
        m = ~np.isnan(w) & (np.abs(w - cut) > 1e-6)
        np.testing.assert_array_equal((g < cut)[m], (w < cut)[m], err_msg=f"{k}<{cut}")
    m = ~np.isnan(want["macd_signal"]) & (np.abs(want["macd"] - want["macd_signal"]) > 1e-9 * np.abs(c))
    np.testing.assert_array_equal((got["macd"] > got["macd_signal"])[m], (want["macd"] > want["macd_signal"])[m])


def test_row_stride_and_rejects_bad_input(cuda):
    panel = numpy_panel(4, 300, seed0=11)
    big = {k: np.concatenate([v, np.zeros((4, 20))], axis=1) for k, v in panel.items()}
    t = {k: torch.from_numpy(v).cuda()[:, :300] for k, v in big.items()}
    out = engine.enrich(t["open"], t["high"], t["low"], t["close"], t["volume"])
    want = ref.enrich_panel(panel["open"], panel["high"], panel["low"], panel["close"], panel["volume"])
    compare({k: v.cpu().numpy() for k, v in out.items()}, want, panel)
    with pytest.raises(ValueError):
        engine.enrich(t["open"].float(), t["high"], t["low"], t["close"], t["volume"])
    with pytest.raises(ValueError):
        engine.enrich(t["open"].cpu(), t["high"], t["low"], t["close"], t["volume"])
    with pytest.raises(ValueError):
        engine.enrich(t["open"], t["high"], t["low"], t["close"], t["volume"],
                      params=engine.IndicatorParams(ma_periods=(7, 25, 500)))


def test_c2_batch_matches_oracle(cuda):
    """BASELINE config C2: 1k symbols x 1k candles (per-symbol price scales
    10^U(-4,4), constant runs, zero-volume bars) against the per-symbol pandas
    oracle, every column, every candle."""
    panel = numpy_panel(1000, 1000, seed0=2026)
    got = run_gpu(panel)
    want = ref.enrich_panel(panel["open"], panel["high"], panel["low"], panel["close"], panel["volume"])
    compare(got, want, panel)


def test_c4_shard_size_properties(cuda):
    """At the C4 shard (12 500 x 10 000, generated in HBM): a sample of rows
    equals the oracle, the NaN warm-up pattern is exact for every row, and
    size-independent identities hold everywhere: bb_mid == ma_20-equivalent
    mean (bb_upper + bb_lower) / 2, macd == ema12 - ema26 sign structure,
    0 <= rsi, mfi <= 100."""
    from binquant_amd.synth import device_panel

    S, T = 12_500, 10_000
    p = device_panel(S, T, seed=77)
    out = engine.enrich(p["open"], p["high"], p["low"], p["close"], p["volume"])
    torch.cuda.synchronize()
    # warm-up NaN prefixes (pandas rolling(w) / min_periods semantics)
    for k, w in (("ma_7", 7), ("ma_25", 25), ("ma_100", 100), ("bb_mid", 20), ("ATR", 14), ("twap", 12),
                 ("rsi", 14), ("mfi", 14)):   # delta.where(...) turns the first NaN into 0
        col = out[k]
        assert torch.isnan(col[:, : w - 1]).all(), k
        assert not torch.isnan(col[:, w:]).any(), k
    for k in ("macd", "macd_signal", "ema20", "ema50"):
        assert not torch.isnan(out[k]).any(), k
    for k in ("rsi", "mfi"):
        v = out[k][:, 20:]
        assert bool(((v >= 0) & (v <= 100)).all()), k
    mid2 = (out["bb_upper"] + out["bb_lower"]) / 2
    rel = ((mid2 - out["bb_mid"]).abs() / out["bb_mid"].abs())[:, 20:]
    assert float(rel.max()) < 1e-12
    # a spread sample of rows against the per-symbol pandas path
    rows = torch.linspace(0, S - 1, 6).long()
    host = {k: v[rows].cpu().numpy() for k, v in p.items()}
    want = ref.enrich_panel(host["open"], host["high"], host["low"], host["close"], host["volume"])
    got = {k: v[rows].cpu().numpy() for k, v in out.items()}
    compare(got, want, host)


def test_padded_output_pitch_is_bit_equal(cuda):
    """engine.enrich_outputs (views of [S, T + 64] buffers on large panels:
    the HBM-friendly row pitch the bench uses, and engine.enrich's own
    default allocation on such panels) gives the same bits as contiguous
    [S, T] outputs; a partial `out` sets the pitch of the columns enrich
    allocates."""
    import numpy as np
    import torch

    from binquant_amd import engine
    from binquant_amd.synth import numpy_panel

    S, T = 1100, 1500
    p = {k: torch.from_numpy(v).cuda() for k, v in numpy_panel(S, T, seed0=9).items()}
    args = [p[k] for k in ("open", "high", "low", "close", "volume")]
    out = engine.enrich_outputs(S, T, "cuda")
    assert next(iter(out.values())).stride(0) == T + engine.ENRICH_ROW_PAD
    a = engine.enrich(*args, out=out)
    flat = {k: torch.empty((S, T), dtype=torch.float64, device="cuda") for k in out}
    b = engine.enrich(*args, out=flat)
    c = engine.enrich(*args)   # default allocation: the padded pitch
    assert all(v.stride(0) == T + engine.ENRICH_ROW_PAD for v in c.values())
    part = engine.enrich(*args, out={"rsi": flat["rsi"]})
    assert all(v.stride(0) == T for v in part.values())
    for k in b:
        np.testing.assert_array_equal(a[k].cpu().numpy(), b[k].cpu().numpy(), err_msg=k)
        np.testing.assert_array_equal(c[k].cpu().numpy(), b[k].cpu().numpy(), err_msg=k)
        np.testing.assert_array_equal(part[k].cpu().numpy(), b[k].cpu().numpy(), err_msg=k)


def test_missing_and_nonfinite_inputs_follow_pandas(cuda):
    """Rows holding NaN or +-inf inputs (a drop-in frame with gaps) take the
    kernel's per-row rewrite (bq_enrich.hip enrich_row_missing): every column
    equals the pandas oracle — windows over a gap NaN, pandas' ewm gap decay
    (bit for bit), SMA RSI / MFI with their where(..., 0.0) rules — while the
    clean rows of the same launch stay on the tile walk (bit-equal to a launch
    of the clean rows alone)."""
    S, T = 12, 2300
    panel = numpy_panel(S, T, seed0=5)
    nan, inf = np.nan, np.inf
    c, h, l, o, v = (panel[k] for k in ("close", "high", "low", "open", "volume"))
    c[1, 500] = nan                                   # one missing close
    for k in (c, h, l, o):
        k[2, 800:806] = nan                           # a missing candle run
    for k in (c, h, l, o, v):
        k[3, :40] = nan                               # a late listing: leading NaN
    v[4, 1200] = inf                                  # inf volume: MFI windows
    c[5, 1500] = inf                                  # inf close (pandas: missing in windows and ewm)
    c[6, 1023:1025] = nan                             # across the 1024-candle tile boundary
    v[7, 300:320] = nan                               # missing volume only
    c[8, -3:] = nan                                   # trailing NaN
    h[9, 100::97] = nan                               # scattered missing highs
    c[10, 0] = nan                                    # missing first close
    got = run_gpu(panel)
    want = ref.enrich_panel(panel["open"], panel["high"], panel["low"], panel["close"], panel["volume"])
    price = np.nanmean(np.where(np.isfinite(c), np.abs(c), np.nan), axis=1, keepdims=True)
    for k in COLS:
        assert_close(got[k], want[k], k, scale=100.0 if k in ("rsi", "mfi") else price)
    for k in ("macd", "macd_signal", "ema20", "ema50"):   # the rewrite replays pandas' recursion
        bad = [s for s in range(1, 11) if not np.array_equal(got[k][s], want[k][s], equal_nan=True)]
        assert not bad, (k, bad)
    clean = {k: v[[0, 11]] for k, v in panel.items()}
    alone = run_gpu(clean)
    for k in COLS:
        np.testing.assert_array_equal(got[k][[0, 11]], alone[k], err_msg=k)
