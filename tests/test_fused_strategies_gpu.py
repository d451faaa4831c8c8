"""The fused strategy passes against the staged pipelines they replace, on
panels with halts, gaps, zero volume and NaN candles:

* bq_pump_features (strategies.pump_score_features, panel mode) — one pass per
  row for every column but the quantiles and score_cross;
* bq_burst_features / bq_burst_qualify (strategies.activity_burst_features)
  — two streaming passes around the score's quantile, bit for bit.

The staged pipelines themselves are pinned to the reference's fixtures
(tests/test_strategies_gpu.py, tests/test_panel_fixtures_gpu.py), which now run
the fused passes too."""

import numpy as np
import pytest
import torch

from tests.util import assert_close

pytestmark = pytest.mark.gpu


def test_pump_fused_equals_staged_panel(cuda):
    """bq_pump_features (one pass per row) against the staged panel pipeline
    on a 200 x 2500 panel with halts, gaps and zero volume: columns whose
    windows are order statistics / shifts equal bit for bit, the volume mean
    and what depends on it within 1e-12 of each row's magnitude (its sliding
    sum restarts at each lane's 4 candles instead of 8), flags equal away
    from near-ties."""
    from binquant_amd import strategies
    from binquant_amd.synth import numpy_panel

    S, T = 200, 2500
    p = numpy_panel(S, T, seed0=31, edges=True)
    p["volume"][3, 700:760] = 0.0
    p["close"][4, 900:905] = np.nan
    d = {k: torch.from_numpy(v).cuda() for k, v in p.items()}
    btc = d["close"][0].clone()
    btc[::17] = float("nan")
    run = lambda: strategies.pump_score_features(d["open"], d["high"], d["low"], d["close"], d["volume"], btc)
    fused = run()
    strategies._PUMP_FUSED = False
    try:
        staged = run()
    finally:
        strategies._PUMP_FUSED = True
    assert list(fused) == list(staged)
    exact_cols = ("candidate_atr", "momentum_3", "pre_breakout_compression", "prior_high", "close_location", "ema20",
                  "ema50", "trend_score", "momentum_atr", "btc_momentum_3", "btc_trend_score", "relative_strength")
    for k in staged:
        x, y = fused[k].cpu().numpy(), staged[k].cpu().numpy()
        if k in exact_cols:
            np.testing.assert_array_equal(x, y, err_msg=k)
        elif y.dtype == bool:
            assert int((x != y).sum()) <= 5, k
        else:
            with np.errstate(all="ignore"):
                fin = np.where(np.isfinite(y), np.abs(y), np.nan)
                sc = np.nan_to_num(np.nanmax(fin, axis=1, initial=0.0), nan=1.0)
            sc = np.where(sc > 0, sc, 1.0)
            assert_close(x, y, f"fused.{k}", rtol=1e-12, scale=np.broadcast_to(sc[:, None], y.shape), atol_rel=1e-13)



@pytest.mark.parametrize("with_q", [True, False])
def test_burst_fused_equals_staged(cuda, with_q):
    from binquant_amd import strategies
    from binquant_amd.synth import numpy_panel

    S, T = 150, 2300
    p = numpy_panel(S, T, seed0=77, edges=True)
    p["volume"][3, 700:760] = 0.0
    p["close"][4, 900:905] = np.nan
    rng = np.random.default_rng(5)
    spikes = rng.random((S, T)) < 0.02   # volume / price bursts so the flags fire
    p["volume"][spikes] *= 8.0
    p["close"][spikes] *= 1.03
    p["high"] = np.fmax(p["high"], p["close"])
    d = {k: torch.from_numpy(v).cuda() for k, v in p.items()}
    qv = d["volume"] * d["close"] if with_q else None
    run = lambda: strategies.activity_burst_features(d["open"], d["high"], d["low"], d["close"], d["volume"], qv)
    fused = run()
    strategies._BURST_FUSED = False
    try:
        staged = run()
    finally:
        strategies._BURST_FUSED = True
    assert list(fused) == list(staged)
    for k in staged:
        x, y = fused[k].cpu().numpy(), staged[k].cpu().numpy()
        assert x.dtype == y.dtype, k
        np.testing.assert_array_equal(x, y, err_msg=k)
    assert staged["qualified_signal"].sum().item() > 0
