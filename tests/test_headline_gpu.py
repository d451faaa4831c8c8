"""GPU parity at the exact configuration bench.py times: BASELINE configs[3],
100 000 symbols x 10 000 candles resident on one GPU, generated in HBM by the
bench's own generator and seed (synth.device_panel(..., seed=1234), rank 0),
ONE engine.enrich launch over the whole panel (grid = 100 000 workgroups,
1e9 candles; producers/context_evaluator.py:240-263 is the call it replaces).

Checked:
* 72 spread rows (symbols 0 and 99 999, the rows whose byte offsets cross
  2^31 and 2^32 — 2^31 / (8 T) = 26 843.5, 2^32 / (8 T) = 53 687.1 — and an
  even spread) against the per-symbol pandas oracle on every candle, the
  partial last 1024-candle tile (candles 9 216 .. 9 999) included; tolerance
  of tests/util.py (1e-9 relative + 1e-11 x price magnitude);
* on EVERY row (1e9 candles per column), as size-independent properties:
  the exact NaN warm-up prefix of each column, rsi / mfi within [0, 100],
  (bb_upper + bb_lower) / 2 == bb_mid to 1e-12, the SMA-family columns
  (ma_7, ma_25, ma_100, bb_mid, twap, ATR) against a torch fp64 window mean
  at 1e-9, bb_upper - bb_mid against torch's ddof-1 window std at 1e-9, and
  pandas' ewm(adjust=False) recursion y_t = (1 - a) y_{t-1} + a x_t holding
  for ema20 / ema50 / macd_signal to 1e-12 of the price magnitude.
"""

from __future__ import annotations

import numpy as np
import pytest
import torch

from binquant_amd import engine
from binquant_amd.synth import device_panel
from oracle import indicators_ref as ref
from tests.test_enrich_gpu import compare

pytestmark = pytest.mark.gpu

S, T = 100_000, 10_000
BENCH_SEED = 1234          # bench.py main(): device_panel(S, T, seed=1234 + rank)
CHUNK = 6_250              # rows per full-panel check (temporaries ~0.5 GB each)


def _sample_rows() -> list[int]:
    edge = [0, 1, 26_842, 26_843, 26_844, 53_686, 53_687, 53_688, 99_998, 99_999]
    spread = np.linspace(0, S - 1, 62).round().astype(int).tolist()
    return sorted(set(edge + spread))


def _window_mean(x: torch.Tensor, w: int) -> torch.Tensor:
    """[n, T] -> [n, T - w + 1]: mean of each length-w window (torch fp64)."""
    return x.unfold(1, w, 1).sum(dim=2) / w


def _assert_rel(got: torch.Tensor, want: torch.Tensor, scale: torch.Tensor, name: str, rtol=1e-9, arel=1e-11):
    err = (got - want).abs()
    lim = rtol * want.abs() + arel * scale
    bad = ~(err <= lim)
    if bool(bad.any()):
        i = int(torch.argmax((err - lim).nan_to_num(nan=float("inf"))).item())
        g, wv = got.reshape(-1)[i].item(), want.reshape(-1)[i].item()
        raise AssertionError(f"{name}: {int(bad.sum())} elements off, e.g. got {g!r} want {wv!r}")


@pytest.fixture(scope="module")
def headline():
    free, total = torch.cuda.mem_get_info()
    need = S * T * 8 * (5 + len(ref.CANONICAL)) + (8 << 30)
    if total < need:
        pytest.skip(f"needs {need / 2**30:.0f} GiB of device memory for the 100k x 10k panel")
    torch.cuda.empty_cache()
    p = device_panel(S, T, seed=BENCH_SEED)
    out = engine.enrich(p["open"], p["high"], p["low"], p["close"], p["volume"])
    torch.cuda.synchronize()
    yield p, out
    del p, out
    torch.cuda.empty_cache()


def test_headline_sampled_rows_match_oracle(headline):
    p, out = headline
    rows = torch.tensor(_sample_rows(), device=p["close"].device)
    host = {k: v[rows].cpu().numpy() for k, v in p.items()}
    got = {k: v[rows].cpu().numpy() for k, v in out.items()}
    want = ref.enrich_panel(host["open"], host["high"], host["low"], host["close"], host["volume"])
    compare(got, want, host)
    # the partial last tile on its own (10 000 = 9 x 1024 + 784), same bar
    tail = slice(9 * 1024, T)
    compare({k: v[:, tail] for k, v in got.items()}, {k: v[:, tail] for k, v in want.items()},
            {k: v[:, tail] for k, v in host.items()})


def test_headline_every_row_properties(headline):
    p, out = headline
    warm = {"ma_7": 6, "ma_25": 24, "ma_100": 99, "bb_mid": 19, "bb_upper": 19, "bb_lower": 19,
            "ATR": 13, "twap": 11, "rsi": 13, "mfi": 13}
    a20, a50, a9 = 2.0 / 21.0, 2.0 / 51.0, 2.0 / 10.0
    for lo in range(0, S, CHUNK):
        hi = min(S, lo + CHUNK)
        c = p["close"][lo:hi]
        o, h, l, v = (p[k][lo:hi] for k in ("open", "high", "low", "volume"))
        col = {k: t[lo:hi] for k, t in out.items()}
        price = c.abs().mean(dim=1, keepdim=True)
        # exact warm-up prefixes: NaN before the first full window, finite after
        # (rsi / mfi: where(delta > 0, 0.0) turns the first NaN diff into 0, so
        # they start at index w - 1 like the means)
        for k, n in warm.items():
            assert bool(torch.isnan(col[k][:, :n]).all()), f"{k}: warm-up not NaN (rows {lo}..{hi})"
            assert not bool(torch.isnan(col[k][:, n:]).any()), f"{k}: NaN after warm-up (rows {lo}..{hi})"
        for k in ("macd", "macd_signal", "ema20", "ema50"):
            assert not bool(torch.isnan(col[k]).any()), k
        for k in ("rsi", "mfi"):
            x = col[k][:, 14:]
            assert bool(((x >= 0) & (x <= 100)).all()), f"{k} outside [0, 100] (rows {lo}..{hi})"
        mid2 = (col["bb_upper"][:, 19:] + col["bb_lower"][:, 19:]) / 2
        assert float(((mid2 - col["bb_mid"][:, 19:]).abs() / col["bb_mid"][:, 19:].abs()).max()) < 1e-12
        # SMA family against torch window means, every candle of every row
        for k, w in (("ma_7", 7), ("ma_25", 25), ("ma_100", 100), ("bb_mid", 20)):
            _assert_rel(col[k][:, w - 1:], _window_mean(c, w), price, f"{k} rows {lo}..{hi}")
        bar = (o + h + l + c) / 4
        _assert_rel(col["twap"][:, 11:], _window_mean(bar, 12), price, f"twap rows {lo}..{hi}")
        del bar
        prev = torch.cat([torch.full_like(c[:, :1], float("nan")), c[:, :-1]], dim=1)
        tr = torch.stack([h - l, (h - prev).abs(), (l - prev).abs()]).nan_to_num(nan=-float("inf")).amax(0)
        del prev
        _assert_rel(col["ATR"][:, 13:], _window_mean(tr, 14), price, f"ATR rows {lo}..{hi}")
        del tr
        sd = c.unfold(1, 20, 1).std(dim=2, unbiased=True)
        _assert_rel(col["bb_upper"][:, 19:] - col["bb_mid"][:, 19:], 2.0 * sd, price, f"bb std rows {lo}..{hi}")
        del sd
        # pandas' ewm(adjust=False) step, checked as a recursion residual
        for k, a, x in (("ema20", a20, c), ("ema50", a50, c), ("macd_signal", a9, col["macd"])):
            y = col[k]
            step = (1.0 - a) * y[:, :-1] + a * x[:, 1:]
            _assert_rel(y[:, 1:], step, price, f"{k} recursion rows {lo}..{hi}", rtol=1e-12, arel=1e-12)
            assert bool((y[:, 0] == x[:, 0]).all()), f"{k}: first value is not the first observation"
        del col
