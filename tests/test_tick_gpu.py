"""GPU parity of the streaming tick path (bq_state_seed + bq_tick) against
the pandas oracle on the full series: tick t must equal row t of
indicators_enrichment over candles [0, t]."""

import numpy as np
import pytest
import torch

from binquant_amd import engine
from binquant_amd.synth import numpy_panel
from oracle import indicators_ref as ref
from tests.util import assert_close

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("S,T0,N", [(64, 400, 60), (8, 1, 130), (300, 150, 5)])
def test_tick_matches_full_series(cuda, S, T0, N):
    T = T0 + N
    panel = numpy_panel(S, T, seed0=S + T)
    want = ref.enrich_panel(panel["open"], panel["high"], panel["low"], panel["close"], panel["volume"])
    dev = {k: torch.from_numpy(v).cuda() for k, v in panel.items()}
    st = engine.TickState(S)
    st.seed(*(dev[k][:, :T0] for k in ("open", "high", "low", "close", "volume")))
    assert st.count == T0
    price = np.abs(panel["close"]).mean(axis=1)
    for t in range(T0, T):
        out = st.tick([dev[k][:, t].contiguous() for k in ("open", "high", "low", "close", "volume")])
        torch.cuda.synchronize()
        for k in ref.CANONICAL:
            scale = 100.0 if k in ("rsi", "mfi") else price
            assert_close(out[k].cpu().numpy(), want[k][:, t], f"{k}@{t}", scale=scale)
    assert st.count == T
    # EMAs are the exact pandas recursion once seeded: bitwise equal
    np.testing.assert_array_equal(out["ema20"].cpu().numpy(), want["ema20"][:, -1])
