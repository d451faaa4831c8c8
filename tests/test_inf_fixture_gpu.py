"""Parity where the strategy frames' rolling windows meet +-inf, against the
REAL reference (tests/golden/inf_windows.npz, tests/golden/make_golden.py
--only inf): 6 symbols x 700 candles with zero-volume halts of 30-60 bars
(the pump's relative_volume = v / 0 = inf after the volume mean's window runs
dry, inside the 48-bar score / volume quantiles) and zero closes (the pct
changes after them are inf, inside the spike pass's 2 / 3 / 5-bar sums and
the |pct change| quantile), every output column of

  a17 ActivityBurstPump.compute_indicators   strategies/activity_burst_pump.py:51-158
  a18 LiquidationSweepPump.compute_pump_score strategies/liquidation_sweep_pump.py:195-269
  a19 FailedSpikeFade.detect                 strategies/failed_spike_fade.py:258-544

at EVERY candle, in the exact (live) mode and the panel mode. pandas' window
operations skip infinities (_prep_values); element-wise columns keep them.
Floats at 1e-9 of the symbol's largest finite magnitude, infinities and NaN
positions equal, flags and labels exactly."""

from pathlib import Path

import numpy as np
import pytest
import torch

from tests.util import assert_close

G = Path(__file__).resolve().parent / "golden"
pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def fx():
    z = np.load(G / "inf_windows.npz")
    d = {k: torch.from_numpy(np.ascontiguousarray(z[k])).cuda()
         for k in ("open", "high", "low", "close", "volume", "qv")}
    return z, d, torch.from_numpy(z["btc_close"]).cuda()


def _check(z, prefix, out, skip=()):
    keys = sorted(k.split("__", 1)[1] for k in z.files if k.startswith(prefix + "__"))
    assert set(keys) <= set(out), sorted(set(keys) - set(out))
    for k in keys:
        if k in skip:
            continue
        g = out[k].cpu().numpy()
        w = z[f"{prefix}__{k}"]
        if g.ndim == 1:
            g = np.broadcast_to(g[:, None], w.shape)
        name = f"{prefix}.{k}"
        if g.dtype == bool:
            np.testing.assert_array_equal(g.astype(float), w, err_msg=name)
            continue
        with np.errstate(all="ignore"):
            fin = np.where(np.isfinite(w), np.abs(w), np.nan)
            sc = np.nan_to_num(np.nanmax(fin, axis=1, initial=0.0), nan=1.0)
        sc = np.where(sc > 0, sc, 1.0)
        assert_close(g, w, name, rtol=1e-9, scale=np.broadcast_to(sc[:, None], w.shape))


@pytest.mark.parametrize("exact", [True, False])
def test_pump_inf_windows(cuda, fx, exact):
    from binquant_amd.strategies import pump_score_features

    z, d, btc = fx
    assert np.isinf(z["lsp__relative_volume"]).any() and np.isinf(z["lsp__pump_score"]).any()
    out = pump_score_features(d["open"], d["high"], d["low"], d["close"], d["volume"], btc, exact=exact)
    _check(z, "lsp", out)


@pytest.mark.parametrize("exact", [True, False])
def test_failed_spike_inf_windows(cuda, fx, exact):
    from binquant_amd.strategies import failed_spike_features

    z, d, _ = fx
    assert np.isinf(z["fsf__price_change"]).any()
    out = failed_spike_features(d["open"], d["high"], d["low"], d["close"], d["volume"], d["qv"], exact=exact)
    _check(z, "fsf", out, skip=("volume_cluster_min_ratio", "price_break_base_threshold"))


def test_activity_burst_inf_windows(cuda, fx):
    from binquant_amd.strategies import activity_burst_features

    z, d, _ = fx
    out = activity_burst_features(d["open"], d["high"], d["low"], d["close"], d["volume"], d["qv"])
    _check(z, "abp", out)
