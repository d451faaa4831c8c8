"""The oracle's restatement of the headline columns against the reference's
own twins at every candle (tests/twins.py; fixtures tests/golden/headline_twins.npz
from the real functions). The GPU kernel is checked against the same fixtures
in tests/test_twins_gpu.py."""

import pandas as pd
import pytest

from oracle import indicators_ref as ref
from tests import twins

FRAMES = twins.load()


def oracle_columns(fr, p):
    """indicators_enrichment over the frame; the two EMA columns under the
    kernel's slot names (ema20 / ema50 hold ema_spans[0] / [1])."""
    df = pd.DataFrame({k: fr[k] for k in ("open", "high", "low", "close", "volume")})
    df = ref.indicators_enrichment(df, dict(p))
    out = {k: df[k].to_numpy() for k in ("ATR", "bb_upper", "bb_mid", "bb_lower", "rsi")}
    out["ema20"] = df[f"ema{p['ema_spans'][0]}"].to_numpy()
    out["ema50"] = df[f"ema{p['ema_spans'][1]}"].to_numpy()
    return out


@pytest.mark.parametrize("name", list(FRAMES))
def test_oracle_matches_reference_twins(name):
    fr = FRAMES[name]
    counts = twins.check_frame(name, fr, oracle_columns(fr, twins.PARAMS_A), oracle_columns(fr, twins.PARAMS_B),
                              exact=True)
    assert min(counts.values()) > 100, counts
