"""bq_enrich against the reference's own twins of the headline columns at
every candle: tests/golden/headline_twins.npz from the
real _compute_symbol_features (EMA 20 / 50, rolling-14 ATR, ddof-0 rolling-20
Bollinger), _compute_rsi (SMA RSI 14 / 6) and _trend_score (EMA 9 / 21 =
price_tracker.py:204-205; 20 / 50), run on every prefix of frames with a
1024-candle tile crossing, a 1e-3 price scale, constant runs and NaN gaps.
The kernel runs with the twins' IndicatorParams (tests/twins.py PARAMS_A / B);
the comparison rules and tolerances are tests/twins.py's. Also the four frames
as ONE ragged launch (rows padded with NaN past their length)."""

import numpy as np
import pytest
import torch

from binquant_amd import engine
from tests import twins

pytestmark = pytest.mark.gpu

FRAMES = twins.load()
FIELDS = ("open", "high", "low", "close", "volume")


def run(panel, p):
    t = [torch.from_numpy(np.ascontiguousarray(panel[k])).cuda() for k in FIELDS]
    out = engine.enrich(*t, params=engine.IndicatorParams(**p))
    torch.cuda.synchronize()
    return {k: v.cpu().numpy() for k, v in out.items()}


@pytest.mark.parametrize("name", list(FRAMES))
def test_enrich_matches_reference_twins(cuda, name):
    fr = FRAMES[name]
    panel = {k: fr[k][None, :] for k in FIELDS}
    a = {k: v[0] for k, v in run(panel, twins.PARAMS_A).items()}
    b = {k: v[0] for k, v in run(panel, twins.PARAMS_B).items()}
    counts = twins.check_frame(name, fr, a, b)
    assert min(counts.values()) > 100, counts


def test_twin_frames_in_one_launch(cuda):
    """The frames side by side in one [4, T_max] launch (the batched call of
    the cohort path), each row checked on its own length."""
    T = max(fr["close"].size for fr in FRAMES.values())
    panel = {k: np.full((len(FRAMES), T), np.nan) for k in FIELDS}
    for i, fr in enumerate(FRAMES.values()):
        for k in FIELDS:
            panel[k][i, : fr[k].size] = fr[k]
    a = run(panel, twins.PARAMS_A)
    b = run(panel, twins.PARAMS_B)
    for i, (name, fr) in enumerate(FRAMES.items()):
        n = fr["close"].size
        twins.check_frame(name, fr, {k: v[i, :n] for k, v in a.items()}, {k: v[i, :n] for k, v in b.items()})
