"""The forward-fill scan (ffill_kernel) against pandas' Series.ffill, and
batches mixing a panel with fewer-row series (bq_roll_job.rows: the [1, T]
benchmark beside an [S, T] panel) against the same series run on their own.
A fill copies values, so both are compared bit for bit."""

import numpy as np
import pandas as pd
import pytest
import torch

from binquant_amd import engine
from binquant_amd.engine import Ewm, Ffill, Roll

pytestmark = pytest.mark.gpu


def _nan_panel(S, T, seed):
    rng = np.random.default_rng(seed)
    x = rng.standard_normal((S, T)) * 10.0 ** rng.uniform(-3, 3, (S, 1))
    x[rng.random((S, T)) < 0.2] = np.nan          # scattered gaps
    x[0, :] = np.nan                                # an all-NaN row
    x[1, : T // 2] = np.nan                         # leading NaNs
    if T > 1100:
        x[2, 900:1100] = np.nan                     # a gap across the 1024-candle tile edge
    x[3, -1] = -0.0                                 # a signed zero carried forward
    x[3, -5:-1] = np.nan
    return x


@pytest.mark.parametrize("T", [1, 5, 1023, 1024, 1025, 2049, 3000])
def test_ffill_scan_matches_pandas(cuda, T):
    x = _nan_panel(6, T, T)
    got = engine.rolling_many(Ffill(torch.from_numpy(x).cuda()))[0].cpu().numpy()
    want = pd.DataFrame(x.T).ffill().to_numpy().T
    np.testing.assert_array_equal(np.isnan(got), np.isnan(want))
    m = ~np.isnan(want)
    assert np.array_equal(got[m].view(np.int64), want[m].view(np.int64)), "ffill must copy values bit for bit"


def test_ffill_strided_rows(cuda):
    x = _nan_panel(5, 1500, 7)
    big = torch.full((5, 1601), float("nan"), dtype=torch.float64, device="cuda")
    big[:, :1500] = torch.from_numpy(x).cuda()
    view = big[:, :1500]                            # row stride 1601: odd, unaligned rows
    got = engine.rolling_many(Ffill(view))[0].cpu().numpy()
    want = pd.DataFrame(x.T).ffill().to_numpy().T
    np.testing.assert_array_equal(got, want)


def test_fewer_row_series_join_the_panel_batch(cuda):
    S, T = 300, 1200
    rng = np.random.default_rng(3)
    panel = torch.from_numpy(100 * np.exp(np.cumsum(rng.normal(0, 0.01, (S, T)), 1))).cuda()
    bench = torch.from_numpy(100 * np.exp(np.cumsum(rng.normal(0, 0.01, (1, T)), 1)))
    bench[0, 17:40] = float("nan")                  # missing benchmark candles
    bench = bench.cuda()
    specs = [Ewm(panel, span=20), Roll(panel, 20, "mean", shift=1), Ffill(panel),
             Ffill(bench), Ewm(bench, span=20), Ewm(bench, span=50), Roll(bench, 12, "std")]
    together = engine.rolling_many(*specs)
    alone = [engine.rolling_many(sp)[0] for sp in specs]
    for i, (a, b) in enumerate(zip(together, alone)):
        assert a.shape == b.shape, i
        assert torch.equal(torch.nan_to_num(a, nan=7.25), torch.nan_to_num(b, nan=7.25)), f"series {i}"
    # and the benchmark EWM is pandas' own (the exact replay)
    want = pd.Series(bench[0].cpu().numpy()).ewm(span=20, adjust=False).mean().to_numpy()
    np.testing.assert_array_equal(together[4][0].cpu().numpy(), want)


def test_fewer_rows_rejected_for_order_statistics(cuda):
    panel = torch.zeros((4, 50), dtype=torch.float64, device="cuda")
    bench = torch.zeros((1, 50), dtype=torch.float64, device="cuda")
    with pytest.raises(ValueError):
        engine.rolling_many(Roll(panel, 5, "mean"), Roll(bench, 5, "median"))
