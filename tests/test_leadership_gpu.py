"""GradualGainerRetest relative-strength leadership on the device
(signals.gradual_gainer_leadership; strategies/gradual_gainer_retest.py:131-196)
against the reference's own outputs on every prefix frame
(tests/golden/leadership.npz, tests/golden/make_golden.py --only leadership):
the frames of the reference's test (tests/test_gradual_gainer_retest.py:13-36)
and a 20 x 360 panel with BTC gaps, a duplicated BTC timestamp, non-positive
closes and a late listing. Booleans exact, relative strengths to 1e-12."""

from pathlib import Path

import numpy as np
import pytest
import torch

from tests.util import assert_close

G = Path(__file__).resolve().parent / "golden"
pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("case", ["ref", "pan"])
def test_leadership_matches_reference(cuda, case):
    from binquant_amd import signals

    z = np.load(G / "leadership.npz")
    d = lambda k: torch.from_numpy(np.ascontiguousarray(z[f"{case}__{k}"])).cuda()  # noqa: E731
    out = signals.gradual_gainer_leadership(d("open_time"), d("close"), d("btc_time"), d("btc_close"))
    np.testing.assert_array_equal(out["leader"].cpu().numpy(), z[f"{case}__leader"])
    for k in ("rs_2h", "rs_6h"):
        assert_close(out[k].cpu().numpy(), z[f"{case}__{k}"], f"{case}.{k}", rtol=1e-12, scale=1.0, atol_rel=1e-15)
    if case == "ref":   # the reference test's own assertion on the last frame
        assert bool(out["leader"][0, -1]) and float(out["rs_2h"][0, -1]) > 0 and float(out["rs_6h"][0, -1]) > 0


def test_leadership_panel_vs_oracle(cuda):
    """a wider panel (300 symbols x 1500 candles, several tiles of the
    order-statistic kernel) against the pandas restatement pinned above"""
    from binquant_amd import signals
    from oracle import indicators_ref

    rng = np.random.default_rng(7)
    S, T = 300, 1500
    t0 = 1_800_000_000_000
    times = np.broadcast_to(t0 + 900_000 * np.arange(T, dtype=np.int64), (S, T)).copy()
    drift = rng.normal(0.0, 0.002, (S, 1))
    close = 10.0 ** rng.uniform(-3, 3, (S, 1)) * np.exp(np.cumsum(rng.normal(0, 0.006, (S, T)) + drift, axis=1))
    keep = rng.random(T) > 0.02
    bt = (t0 + 900_000 * np.arange(T, dtype=np.int64))[keep]
    bc = 30_000.0 * np.exp(np.cumsum(rng.normal(0, 0.004, keep.sum())))
    want = indicators_ref.gradual_gainer_leadership(times, close, bt, bc)
    tt = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda()  # noqa: E731
    out = signals.gradual_gainer_leadership(tt(times), tt(close), tt(bt), tt(bc))
    np.testing.assert_array_equal(out["leader"].cpu().numpy(), want[0])
    assert want[0].sum() > 100
    np.testing.assert_array_equal(out["rs_2h"].cpu().numpy(), want[1])
    np.testing.assert_array_equal(out["rs_6h"].cpu().numpy(), want[2])


@pytest.mark.parametrize("S,T,bench_gaps", [(300, 1500, True), (7, 2500, True), (3, 97, True), (64, 2600, False),
                                             (5, 300, False)])
def test_leadership_fused_equals_staged(cuda, S, T, bench_gaps):
    """bq_leadership (one counting pass) against the staged pipeline (align, fused
    stages, the order-statistic jobs, the integer rolling sum) bit for bit:
    BTC gaps and a duplicated BTC time, zero / negative closes, a late
    listing, symbols on their own time grids; T = 2500 at 7 symbols runs
    several 256-candle tiles per row (each with its 95-entry history halo).
    Without BTC gaps every row sits on the benchmark's grid and reads the
    benchmark's shared strength ratios, but the rows given a gap of their
    own (a skipped candle, a two-hour hole) divide again in the tiles that
    hold the gap."""
    from binquant_amd import signals

    rng = np.random.default_rng(S * 7 + T)
    t0 = 1_800_000_000_000
    grid = t0 + 900_000 * np.arange(T + 40, dtype=np.int64)
    off = rng.integers(0, 40, S)
    times = np.stack([grid[o:o + T] for o in off])
    close = 10.0 ** rng.uniform(-3, 3, (S, 1)) * np.exp(np.cumsum(rng.normal(0, 0.006, (S, T)), axis=1))
    close[0, 500 % T:520 % T] = 0.0
    close[1 % S, 700 % T] = -1.0
    close[2 % S, : T // 3] = 0.0   # late listing
    if bench_gaps:
        keep = rng.random(T + 40) > 0.03
        bt = grid[keep]
        bt = np.sort(np.concatenate([bt, bt[5:6]]))   # a duplicated time: the later row wins
    else:
        bt = np.concatenate([grid, grid[-1] + 900_000 * np.arange(1, 41, dtype=np.int64)])
        times[3 % S, T // 2:] += 900_000        # a skipped candle
        times[4 % S, T // 3:] += 8 * 900_000    # a two-hour hole
    bc = 30_000.0 * np.exp(np.cumsum(rng.normal(0, 0.004, bt.size)))
    tt = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda()  # noqa: E731
    for q in (0.80, 0.55):   # the strategy's RS_QUANTILE and another (the count test holds for any q)
        fused = signals.gradual_gainer_leadership(tt(times), tt(close), tt(bt), tt(bc), rs_quantile=q)
        signals._LEADERSHIP_FUSED = False
        try:
            staged = signals.gradual_gainer_leadership(tt(times), tt(close), tt(bt), tt(bc), rs_quantile=q)
        finally:
            signals._LEADERSHIP_FUSED = True
        for k in ("leader", "rs_2h", "rs_6h"):
            np.testing.assert_array_equal(fused[k].cpu().numpy(), staged[k].cpu().numpy(), err_msg=f"{k} q={q}")
        assert T < 200 or fused["leader"].sum().item() > 0


def test_leadership_other_parameters_stage(cuda):
    """parameters other than the compiled ones (lookback 48) run the staged
    pipeline: engine.leadership declines them"""
    from binquant_amd import engine, signals

    z = np.load(G / "leadership.npz")
    d = lambda k: torch.from_numpy(np.ascontiguousarray(z[f"pan__{k}"])).cuda()  # noqa: E731
    assert engine.leadership(d("open_time"), d("close"), d("btc_time"), d("btc_close"), lookback=48) is None
    out = signals.gradual_gainer_leadership(d("open_time"), d("close"), d("btc_time"), d("btc_close"),
                                            rs_lookback=48)
    assert out["leader"].dtype == torch.bool and out["rs_2h"].shape == d("close").shape
