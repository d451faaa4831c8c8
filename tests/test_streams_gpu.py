"""Launch ordering of the public entry points (engine.launch_scope): a call
with `stream=` on a side stream waits for the producers of its operands on the
current stream, allocates and computes on the side stream, and keeps the
operands alive for it; results equal the current-stream call bit for bit."""

import pytest
import torch

from binquant_amd import engine
from binquant_amd import fused as F
from binquant_amd.synth import device_panel

pytestmark = pytest.mark.gpu


def test_side_stream_enrich_and_fused_match_current_stream(cuda):
    p = device_panel(300, 3000, seed=2)
    want = engine.enrich(p["open"], p["high"], p["low"], p["close"], p["volume"])
    want_f = F.run({"r": (F.inp(p["close"]) - F.inp(p["open"])) / F.inp(p["open"])})["r"]
    side = torch.cuda.Stream()
    for _ in range(3):
        # operands produced on the current stream right before the call
        c = p["close"] * 1.0
        o = p["open"] * 1.0
        got = engine.enrich(o, p["high"], p["low"], c, p["volume"], stream=side)
        got_f = F.run({"r": (F.inp(c) - F.inp(o)) / F.inp(o)}, stream=side)["r"]
        del c, o   # freed on the current stream while the side stream may still read them
        torch.cuda.current_stream().wait_stream(side)
        for k, v in want.items():
            assert torch.equal(torch.nan_to_num(got[k], nan=7.0), torch.nan_to_num(v, nan=7.0)), k
        assert torch.equal(got_f, want_f)


def test_side_stream_tick_and_features(cuda):
    p = device_panel(500, 420, seed=9)
    st_a, st_b = engine.TickState(500), engine.TickState(500)
    st_a.seed(*(p[k][:, :400] for k in ("open", "high", "low", "close", "volume")))
    side = torch.cuda.Stream()
    st_b.seed(*(p[k][:, :400] for k in ("open", "high", "low", "close", "volume")), stream=side)
    for t in range(400, 420):
        new = [p[k][:, t].contiguous() for k in ("open", "high", "low", "close", "volume")]
        a = st_a.tick(new)
        b = st_b.tick(new, stream=side)
        torch.cuda.current_stream().wait_stream(side)
        for k in a:
            assert torch.equal(torch.nan_to_num(a[k], nan=7.0), torch.nan_to_num(b[k], nan=7.0)), (k, t)
    fa = engine.market_features(p["high"], p["low"], p["close"])
    fb = engine.market_features(p["high"], p["low"], p["close"], stream=side)
    torch.cuda.current_stream().wait_stream(side)
    for k in fa:
        assert torch.equal(torch.nan_to_num(fa[k], nan=7.0), torch.nan_to_num(fb[k], nan=7.0)), k


def test_operands_on_two_devices_are_rejected(cuda):
    p = device_panel(4, 100, seed=1)
    with pytest.raises(ValueError):
        engine.enrich(p["open"], p["high"], p["low"], p["close"], p["volume"].cpu())
    st = engine.TickState(4)
    with pytest.raises(ValueError):
        st.tick([p[k][:, 0].cpu() for k in ("open", "high", "low", "close", "volume")])
