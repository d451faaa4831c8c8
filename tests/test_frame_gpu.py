"""GPU parity of the frame plumbing (bq_frame.hip) vs pandas (oracle/frame_ref.py):
resample (Candles.resample, context_evaluator.py:403-407), the benchmark left
merge (liquidation_sweep_pump.py:255-263) and the inner-joined return pairs +
rolling beta/corr (context_evaluator.py:161-194). Resample/merge are exact
(bit-for-bit: comparisons, copies and pandas' Kahan sum replayed); beta/corr
use the 1e-9 fp64 tolerance of tests/util.py."""

import numpy as np
import pandas as pd
import pytest
import torch

from binquant_amd import engine
from binquant_amd.candles import RESAMPLE_AGG, Candles, resample_frames
from binquant_amd.synth import numpy_symbol
from oracle import frame_ref as fref
from tests.util import assert_close

pytestmark = pytest.mark.gpu

M15 = 900_000


def kline_frame(n, seed, start=1_700_000_123_000 // M15 * M15, drop=0.1, nan=0.02):
    rng = np.random.default_rng(seed)
    t = start + M15 * np.arange(int(n * 1.3))
    t = np.sort(rng.choice(t, size=n, replace=False)) if n else t[:0]   # gaps -> short / empty bins
    sym = numpy_symbol(max(n, 1), seed)
    df = pd.DataFrame({k: sym[k][:n] for k in ("open", "high", "low", "close", "volume")})
    df.insert(0, "open_time", t)
    df["close_time"] = t + M15 - 1
    df["quote_asset_volume"] = df["volume"] * df["close"]
    df["number_of_trades"] = rng.integers(0, 50, n).astype(float)
    for c in ("volume", "close", "high"):
        df.loc[rng.random(n) < nan, c] = np.nan
    return df


def assert_frame_equal_exact(got: pd.DataFrame, want: pd.DataFrame):
    assert len(got) == len(want)
    np.testing.assert_array_equal(got["open_time"].to_numpy(), want["open_time"].to_numpy())
    for c in want.columns:
        if c == "open_time":
            continue
        g, w = got[c].to_numpy(np.float64), want[c].to_numpy(np.float64)
        np.testing.assert_array_equal(np.isnan(g), np.isnan(w), err_msg=c)
        m = ~np.isnan(w)
        np.testing.assert_array_equal(g[m], w[m], err_msg=c)


@pytest.mark.parametrize("interval", ["1h", "4h", "30min"])
def test_resample_ragged_frames_match_pandas(cuda, interval):
    frames = [kline_frame(n, 11 * n + 3) for n in (0, 1, 2, 5, 97, 400, 1201)]
    got = resample_frames(frames, interval)
    for df, g in zip(frames, got):
        if len(df) == 0:
            assert len(g) == 0
            continue
        want = fref.resample(df, interval, RESAMPLE_AGG)
        assert_frame_equal_exact(g, want[list(g.columns)])


def test_candles_resample_api(cuda):
    df = Candles(exchange="binance", candles=[]).ensure_ohlc(kline_frame(300, 7, nan=0.0))
    g = Candles(exchange="binance").resample(df, interval="1h")
    want = fref.resample(df, "1h", RESAMPLE_AGG)
    assert_frame_equal_exact(g, want[list(g.columns)])
    assert isinstance(g.index, pd.DatetimeIndex)


def test_resample_kahan_sum_bitwise(cuda):
    """Signed heavy-tailed volumes: ~5% of 4-candle bins have a naive sum that
    differs from pandas' compensated group_sum in the last bits."""
    n = 4000
    rng = np.random.default_rng(1)
    t = (1_700_000_000_000 // 3_600_000) * 3_600_000 + M15 * np.arange(n)
    v = rng.lognormal(3, 2, n) * rng.choice([1.0, -1.0], n)
    df = pd.DataFrame({"open_time": t, "volume": v})
    ts = torch.from_numpy(t[None]).cuda()
    _, outs, nb = engine.resample(ts, {"volume": torch.from_numpy(v[None]).cuda()}, {"volume": "sum"}, 3_600_000)
    want = fref.resample(df, "1h", {"volume": "sum"})["volume"].to_numpy()
    np.testing.assert_array_equal(outs["volume"][0, : int(nb[0])].cpu().numpy(), want)


def test_align_left_merge_matches_pandas(cuda):
    rng = np.random.default_rng(3)
    base = 1_700_000_000_000
    S, T = 9, 300
    ts = base + M15 * np.sort(np.stack([rng.choice(400, T, replace=False) for _ in range(S)]), axis=1)
    bts = base + M15 * np.sort(np.r_[rng.choice(400, 250, replace=False), [5, 5, 17]])   # duplicates
    bval = rng.random(bts.size) * 100
    lens = np.array([T, 0, 1, 17, T, 200, 299, T, 64])
    out = engine.align(torch.from_numpy(ts).cuda(), torch.from_numpy(bts).cuda(), torch.from_numpy(bval).cuda(),
                       lens=lens).cpu().numpy()
    for s in range(S):
        n = lens[s]
        want = fref.left_merge(ts[s, :n], bts, bval)
        np.testing.assert_array_equal(out[s, :n], want)
        assert np.isnan(out[s, n:]).all()


@pytest.mark.parametrize("window", [50, 20])
def test_joined_returns_and_beta_corr_match_reference(cuda, window):
    rng = np.random.default_rng(window)
    base = 1_700_000_000_000
    S, T = 6, 700
    bts = base + M15 * np.sort(rng.choice(900, 800, replace=False))
    bclose = 30000 * np.exp(np.cumsum(rng.normal(0, 0.003, bts.size)))
    ts = base + M15 * np.sort(np.stack([rng.choice(900, T, replace=False) for _ in range(S)]), axis=1)
    close = 10 * np.exp(np.cumsum(rng.normal(0, 0.004, (S, T)), axis=1))
    lens = np.array([T, 40, 0, 500, T, 2])
    x, y, n = engine.join_returns(torch.from_numpy(ts).cuda(), torch.from_numpy(close).cuda(),
                                  torch.from_numpy(bts).cuda(), torch.from_numpy(bclose).cuda(), lens=lens)
    bc = engine.beta_corr_pairs(x, y, window)
    x, y, n = x.cpu().numpy(), y.cpu().numpy(), n.cpu().numpy()
    beta, corr = bc["beta"].cpu().numpy(), bc["corr"].cpu().numpy()
    for s in range(S):
        r = fref.joined_returns(ts[s, : lens[s]], close[s, : lens[s]], bts, bclose)
        k = len(r)
        assert n[s] == k
        assert_close(x[s, :k], r["alt"].to_numpy(), f"alt[{s}]", rtol=1e-14)
        assert_close(y[s, :k], r["btc"].to_numpy(), f"btc[{s}]", rtol=1e-14)
        if k:
            wb, wc = fref.beta_corr_series(r, window)
            assert_close(beta[s, :k], wb, f"beta[{s}]", rtol=1e-9, scale=np.nanmax(np.abs(wb)) if k >= window else 1.0)
            assert_close(corr[s, :k], wc, f"corr[{s}]", rtol=1e-9, scale=1.0)


def test_dynamic_btc_beta_corr_on_timestamp_index(cuda):
    """The scalar drop-in on frames with different gaps (rows joined by
    open_time, not by position)."""
    from binquant_amd.indicators import dynamic_btc_beta_corr_frames

    rng = np.random.default_rng(9)
    base = 1_700_000_000_000
    bts = base + M15 * np.arange(300)
    bclose = 30000 * np.exp(np.cumsum(rng.normal(0, 0.003, 300)))
    keep = np.sort(rng.choice(300, 240, replace=False))
    close = 5 * np.exp(np.cumsum(rng.normal(0, 0.004, 240)))
    df = pd.DataFrame({"open_time": bts[keep], "close": close})
    df_btc = pd.DataFrame({"open_time": bts, "close": bclose})
    beta, corr = dynamic_btc_beta_corr_frames([df], df_btc, window=50, decimals=None)[0]
    r = fref.joined_returns(bts[keep], close, bts, bclose)
    wb, wc = fref.beta_corr_series(r, 50)
    assert abs(beta - wb[-1]) <= 1e-9 * abs(wb[-1]) and abs(corr - wc[-1]) <= 1e-9


@pytest.mark.parametrize("T", [2048, 3000, 4096, 5000])
@pytest.mark.parametrize("dup", [0, 1, 3])
def test_joined_returns_long_rows(cuda, T, dup):
    """Rows on the benchmark's 15-minute grid (the index guess hits) with
    missing candles on both sides, a zero close and `dup` extra copies of one
    benchmark time (pandas' inner join, context_evaluator.py:171-175, joins a
    candle to every copy, each with the return over the row before it), at
    the lengths that pick the whole-row kernel with 8 / 16 candles per thread
    (T <= 2 048 / 4 096) and the tiled kernel (T > 4 096): the oracle's joined
    returns, element for element."""
    rng = np.random.default_rng(T + dup)
    base = 1_700_000_000_000
    nb = 3 * T + 300
    d = 2 * T + 100                                      # the repeated time, past every whole-row span
    grid = base + M15 * np.arange(nb)
    keepb = np.ones(nb, bool)
    keepb[rng.choice(np.r_[0:d, d + 1:nb], 20, replace=False)] = False
    bts = np.sort(np.r_[grid[keepb], np.full(dup, grid[d])])
    bclose = 30000 * np.exp(np.cumsum(rng.normal(0, 0.003, bts.size)))
    S = 4
    ts = np.stack([base + M15 * (np.arange(T) + 17 * s) for s in range(S)])
    for s in range(1, S):   # gaps in the symbol rows too
        drop = rng.choice(T, 10, replace=False)
        row = np.delete(ts[s], drop)
        ts[s] = np.r_[row, row[-1] + M15 * np.arange(1, 11)]
    # row 0 jumps to the repeated time (the guess misses, the search finds
    # it); row 3 starts just before it (its guessed span holds it)
    h = T // 2
    ts[0, h:] = grid[d - 5] + M15 * np.arange(T - h)
    ts[3] = grid[d - T // 4] + M15 * np.arange(T)
    close = 10 * np.exp(np.cumsum(rng.normal(0, 0.004, (S, T)), axis=1))
    close[2, T // 3] = 0.0
    lens = np.array([T, T, T - 5, T // 2])
    x, y, n = engine.join_returns(torch.from_numpy(ts).cuda(), torch.from_numpy(close).cuda(),
                                  torch.from_numpy(bts).cuda(), torch.from_numpy(bclose).cuda(), lens=lens)
    x, y, n = x.cpu().numpy(), y.cpu().numpy(), n.cpu().numpy()
    for s in range(S):
        r = fref.joined_returns(ts[s, : lens[s]], close[s, : lens[s]], bts, bclose)
        k = len(r)
        assert n[s] == k, (s, n[s], k)
        assert_close(x[s, :k], r["alt"].to_numpy(), f"alt[{s}]", rtol=1e-14)
        assert_close(y[s, :k], r["btc"].to_numpy(), f"btc[{s}]", rtol=1e-14)
        assert np.isnan(x[s, k:]).all() and np.isnan(y[s, k:]).all()


def test_joined_returns_capacity(cuda):
    """Every benchmark time held three times: a row joins up to 3 (T - 1)
    pairs. The default capacity (None) sizes the output from the rows'
    benchmark multiplicities and holds all of them; a fixed capacity of T
    cuts the row at T pairs (the oracle's first T); the drop-in
    dynamic_btc_beta_corr_frames sizes it exactly itself."""
    from binquant_amd.indicators import dynamic_btc_beta_corr_frames

    rng = np.random.default_rng(5)
    base = 1_700_000_000_000
    T, nb = 120, 150
    bts = np.repeat(base + M15 * np.arange(nb), 3)
    bclose = 30000 * np.exp(np.cumsum(rng.normal(0, 0.003, bts.size)))
    ts = (base + M15 * (np.arange(T) + 7))[None]
    close = 10 * np.exp(np.cumsum(rng.normal(0, 0.004, (1, T)), axis=1))
    r = fref.joined_returns(ts[0], close[0], bts, bclose)
    k = len(r)
    assert k > T
    args = (torch.from_numpy(ts).cuda(), torch.from_numpy(close).cuda(), torch.from_numpy(bts).cuda(),
            torch.from_numpy(bclose).cuda())
    x, y, n = engine.join_returns(*args, capacity=T)
    assert x.shape == (1, T) and int(n[0]) == T
    assert_close(x[0].cpu().numpy(), r["alt"].to_numpy()[:T], "alt cut", rtol=1e-14)
    assert_close(y[0].cpu().numpy(), r["btc"].to_numpy()[:T], "btc cut", rtol=1e-14)
    x, y, n = engine.join_returns(*args)
    cap = x.shape[1]
    assert cap == 3 * (T - 1) and int(n[0]) == k
    assert_close(x[0, :k].cpu().numpy(), r["alt"].to_numpy(), "alt", rtol=1e-14)
    assert_close(y[0, :k].cpu().numpy(), r["btc"].to_numpy(), "btc", rtol=1e-14)
    assert torch.isnan(x[0, k:]).all() and torch.isnan(y[0, k:]).all()
    df = pd.DataFrame({"open_time": ts[0], "close": close[0]})
    df_btc = pd.DataFrame({"open_time": bts, "close": bclose})
    beta, corr = dynamic_btc_beta_corr_frames([df], df_btc, window=50, decimals=None)[0]
    wb, wc = fref.beta_corr_series(r, 50)
    assert abs(beta - wb[-1]) <= 1e-9 * abs(wb[-1]) and abs(corr - wc[-1]) <= 1e-9


def test_joined_returns_many_to_many(cuda):
    """a frame repeating its own open_time k_l times against a
    benchmark time held k_r times joins k_l * k_r pairs (pandas'
    many-to-many inner join). The default capacity holds them all, and the
    drop-in's beta / corr at the last joined row equals the oracle's."""
    from binquant_amd.indicators import dynamic_btc_beta_corr_frames

    rng = np.random.default_rng(9)
    base = 1_700_000_000_000
    nb, T = 160, 140
    bt = base + M15 * np.arange(nb)
    bts = np.sort(np.r_[bt, bt[40:60], bt[40:50], bt[-3:]])
    bclose = 30000 * np.exp(np.cumsum(rng.normal(0, 0.003, bts.size)))
    own = base + M15 * (np.arange(T) + 10)
    ts = np.sort(np.r_[own, own[35:45], own[-2:]])[None]
    close = 10 * np.exp(np.cumsum(rng.normal(0, 0.004, ts.shape), axis=1))
    r = fref.joined_returns(ts[0], close[0], bts, bclose)
    k = len(r)
    x, y, n = engine.join_returns(torch.from_numpy(ts).cuda(), torch.from_numpy(close).cuda(),
                                  torch.from_numpy(bts).cuda(), torch.from_numpy(bclose).cuda())
    assert int(n[0]) == k and x.shape[1] >= k > ts.shape[1]
    assert_close(x[0, :k].cpu().numpy(), r["alt"].to_numpy(), "alt", rtol=1e-14)
    assert_close(y[0, :k].cpu().numpy(), r["btc"].to_numpy(), "btc", rtol=1e-14)
    df = pd.DataFrame({"open_time": ts[0], "close": close[0]})
    df_btc = pd.DataFrame({"open_time": bts, "close": bclose})
    beta, corr = dynamic_btc_beta_corr_frames([df], df_btc, window=50, decimals=None)[0]
    wb, wc = fref.beta_corr_series(r, 50)
    assert abs(beta - wb[-1]) <= 1e-9 * abs(wb[-1]) and abs(corr - wc[-1]) <= 1e-9
