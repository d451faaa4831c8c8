"""a11/a12: rolling BTC beta/correlation and the BTC 24h change vs the
reference's own values (tests/golden/beta_corr.npz) and the oracle."""

from pathlib import Path

import numpy as np
import pandas as pd
import pytest
import torch

from oracle import indicators_ref as ref
from tests.util import assert_close

G = Path(__file__).resolve().parent / "golden"
CASES = ("corr_pos", "corr_neg", "short")


@pytest.mark.parametrize("case", CASES)
def test_oracle_matches_reference_golden(case):
    z = np.load(G / "beta_corr.npz")
    c, b = z[f"{case}__close"], z[f"{case}__btc"]
    beta, corr = ref.beta_corr_series(c, b, 50)
    want_b, want_c = z[f"{case}__beta_last"], z[f"{case}__corr_last"]
    got_b = np.where(np.isnan(beta), 0.0, beta)
    got_c = np.where(np.isnan(corr), 0.0, corr)
    got_b[np.arange(len(c)) < 50] = 0.0
    got_c[np.arange(len(c)) < 50] = 0.0
    np.testing.assert_allclose(got_b[1:], want_b[1:], rtol=1e-12, atol=1e-15)
    np.testing.assert_allclose(got_c[1:], want_c[1:], rtol=1e-12, atol=1e-15)
    chg = pd.Series(b).pct_change(periods=96).to_numpy() * 100
    np.testing.assert_allclose(chg, z[f"{case}__btc_change_96"], rtol=0, atol=0, equal_nan=True)


@pytest.mark.gpu
@pytest.mark.parametrize("case", CASES)
def test_kernel_matches_reference_golden(cuda, case):
    from binquant_amd import engine

    z = np.load(G / "beta_corr.npz")
    c, b = z[f"{case}__close"], z[f"{case}__btc"]
    out = engine.beta_corr(torch.from_numpy(c)[None].cuda(), torch.from_numpy(b).cuda(), window=50)
    beta = out["beta"][0].cpu().numpy()
    corr = out["corr"][0].cpu().numpy()
    want_b, want_c = z[f"{case}__beta_last"], z[f"{case}__corr_last"]
    t = np.arange(len(c))
    assert np.isnan(beta[t < 50]).all() and np.isnan(corr[t < 50]).all()
    m = t >= 50
    assert_close(np.nan_to_num(beta[m]), want_b[m], "beta", rtol=1e-9, scale=1.0)
    assert_close(np.nan_to_num(corr[m]), want_c[m], "corr", rtol=1e-9, scale=1.0)


@pytest.mark.gpu
def test_kernel_panel_matches_oracle_multi_tile(cuda):
    from binquant_amd import engine
    from binquant_amd.synth import numpy_panel

    S, T = 24, 2600
    p = numpy_panel(S, T, seed0=77, edges=True)
    btc = p["close"][0].copy()
    out = engine.beta_corr(torch.from_numpy(p["close"]).cuda(), torch.from_numpy(btc).cuda(), window=50)
    for s in range(S):
        wb, wc = ref.beta_corr_series(p["close"][s], btc, 50)
        assert_close(out["beta"][s].cpu().numpy(), wb, f"beta[{s}]", rtol=1e-8, scale=1.0)
        assert_close(out["corr"][s].cpu().numpy(), wc, f"corr[{s}]", rtol=1e-8, scale=1.0)


@pytest.mark.gpu
def test_dropin_scalar(cuda):
    from binquant_amd.indicators import btc_price_change, dynamic_btc_beta_corr

    z = np.load(G / "beta_corr.npz")
    for case in CASES:
        c, b = z[f"{case}__close"], z[f"{case}__btc"]
        beta, corr = dynamic_btc_beta_corr(pd.DataFrame({"close": c}), pd.DataFrame({"close": b}), decimals=None)
        assert beta == pytest.approx(z[f"{case}__beta_last"][-1], rel=1e-9, abs=1e-12)
        assert corr == pytest.approx(z[f"{case}__corr_last"][-1], rel=1e-9, abs=1e-12)
        assert btc_price_change(pd.DataFrame({"close": b})) == pytest.approx(
            z[f"{case}__btc_change_96"][-1], nan_ok=True)


@pytest.mark.gpu
@pytest.mark.parametrize("window", [5, 50, 126])
@pytest.mark.parametrize("odd_stride", [False, True])
def test_kernel_jumps_partial_tiles_and_strides(cuda, window, odd_stride):
    """Moves beyond the kernel's short-ratio log path (|c/p - 1| > 1/8: the
    library log), ragged last tiles, the largest window, and rows whose
    stride rules out the 16-byte accesses (odd leading dimension). (Window 2
    is left out: on the self pair its covariance cancels to ~1e-7 relative in
    pandas itself, below any fixed tolerance.)"""
    from binquant_amd import engine

    rng = np.random.default_rng(window + 7 * odd_stride)
    S, T = 6, 1337
    r = rng.normal(0.0, 0.01, size=(S, T))
    jumps = rng.random((S, T)) < 0.02
    r[jumps] = rng.choice([-0.4, -0.15, 0.14, 0.5], size=int(jumps.sum()))
    close = 50.0 * np.exp(np.cumsum(r, axis=1))
    close[2, 400:480] = close[2, 399]   # a halted stretch: zero returns
    btc = close[0].copy()
    ld = T + 1 if odd_stride else T
    buf = torch.zeros((S, ld), dtype=torch.float64, device="cuda")
    buf[:, :T] = torch.from_numpy(close).cuda()
    out = engine.beta_corr(buf[:, :T], torch.from_numpy(btc).cuda(), window=window)
    for s in range(S):
        wb, wc = ref.beta_corr_series(close[s], btc, window)
        assert_close(out["beta"][s].cpu().numpy(), wb, f"beta[{s}]", rtol=1e-8, scale=1.0)
        assert_close(out["corr"][s].cpu().numpy(), wc, f"corr[{s}]", rtol=1e-8, scale=1.0)


@pytest.mark.gpu
def test_entry_points_agree(cuda):
    """bq_beta_corr_ws (engine), bq_beta_corr_bret (benchmark returns given)
    and bq_beta_corr (both price rows, returns formed per wave) compute the
    same sums: equal to 1e-12 on a panel with halts and jumps."""
    import ctypes

    from binquant_amd import _lib, engine
    from binquant_amd.synth import numpy_panel

    S, T, w = 20, 1500, 50
    p = numpy_panel(S, T, seed0=5, edges=True)
    c = torch.from_numpy(np.ascontiguousarray(p["close"])).cuda()
    b = c[3].clone()
    ref_out = engine.beta_corr(c, b, w)
    lib = _lib.load()
    vp = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
    beta0, corr0 = torch.empty_like(c), torch.empty_like(c)
    _lib.check(lib.bq_beta_corr(vp(c), vp(b), S, T, T, w, vp(beta0), vp(corr0), T, None), "bq_beta_corr")
    bret = torch.full((T,), float("nan"), dtype=torch.float64, device="cuda")
    torch.log(b[1:] / b[:-1], out=bret[1:])
    scratch = torch.empty(3 * T, dtype=torch.float64, device="cuda")
    beta3, corr3 = torch.empty_like(c), torch.empty_like(c)
    _lib.check(lib.bq_beta_corr_bret(vp(c), vp(bret), vp(scratch), S, T, T, w, vp(beta3), vp(corr3), T, None),
               "bq_beta_corr_bret")
    torch.cuda.synchronize()
    for got in (beta0, beta3):
        assert_close(got.cpu().numpy(), ref_out["beta"].cpu().numpy(), "beta", rtol=1e-12, scale=1.0)
    for got in (corr0, corr3):
        assert_close(got.cpu().numpy(), ref_out["corr"].cpu().numpy(), "corr", rtol=1e-12, scale=1.0)


@pytest.mark.gpu
@pytest.mark.parametrize("T", [1, 2, 50, 51, 255, 256, 257, 384, 512, 513])
def test_kernel_tile_edges(cuda, T):
    """Row lengths around the wave walker's 256-candle tiles and the window
    (first full window at t = w; the halo re-based at every tile end)."""
    from binquant_amd import engine
    from binquant_amd.synth import numpy_panel

    S, w = 5, 50
    p = numpy_panel(S, max(T, 2), seed0=T, edges=True)
    close = np.ascontiguousarray(p["close"][:, :T])
    btc = close[1].copy()
    out = engine.beta_corr(torch.from_numpy(close).cuda(), torch.from_numpy(btc).cuda(), window=w)
    for s in range(S):
        wb, wc = ref.beta_corr_series(close[s], btc, w)
        assert_close(out["beta"][s].cpu().numpy(), wb, f"beta[{s}]", rtol=1e-8, scale=1.0)
        assert_close(out["corr"][s].cpu().numpy(), wc, f"corr[{s}]", rtol=1e-8, scale=1.0)


# ---- a12: the BTC 24h change with pandas' default pad fill -----------------
def _btc_change_cases():
    z = np.load(G / "btc_change.npz")
    names = sorted({k.split("__")[0] for k in z.files})
    return z, names


def test_pct_change_pad_oracle_matches_pandas_fixture():
    """oracle.pct_change_pad == pandas 2.3.3's pct_change(96) (default pad
    fill) on every case of tests/golden/btc_change.npz, bit for bit."""
    z, names = _btc_change_cases()
    assert len(names) == 12
    for n in names:
        got = ref.pct_change_pad(z[f"{n}__close"], 96) * 100
        np.testing.assert_array_equal(got, z[f"{n}__pct"], err_msg=n)
        np.testing.assert_array_equal(got[-1:], np.atleast_1d(z[f"{n}__last"]), err_msg=n)


@pytest.mark.gpu
def test_btc_change_pad_fill_matches_pandas_fixture(cuda):
    """a12 on the device, bit for bit against pandas' own values: the [S, T]
    engine.pct_change over all 400-candle cases in one panel, the drop-in
    btc_price_change per frame, and the message cohort's btc.change_24h
    stage (cohort.py) — NaN at the last row / at t - 96 / across both,
    leading NaNs, short frames, a zero close."""
    from binquant_amd import engine
    from binquant_amd.indicators import btc_price_change

    z, names = _btc_change_cases()
    full = [n for n in names if z[f"{n}__close"].size == 400]
    panel = torch.from_numpy(np.stack([z[f"{n}__close"] for n in full])).cuda()
    got = (engine.pct_change(panel, 96) * 100).cpu().numpy()
    for i, n in enumerate(full):
        np.testing.assert_array_equal(got[i], z[f"{n}__pct"], err_msg=n)
    for n in names:
        v = btc_price_change(pd.DataFrame({"close": z[f"{n}__close"]}))
        want = float(z[f"{n}__last"])
        assert (np.isnan(v) and np.isnan(want)) or v == want, (n, v, want)
    raw = (engine.pct_change(panel, 96, fill_method=None) * 100).cpu().numpy()
    i = full.index("nan_t96")
    assert np.isnan(raw[i, -1]) and not np.isnan(got[i, -1])
