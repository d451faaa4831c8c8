"""hipGraph replay of the strategy pipelines (binquant_amd.graphs): a replay
equals the eager call bit for bit, also after new inputs are copied in."""

import pytest
import torch

pytestmark = pytest.mark.gpu


def _equal(a, b, where):
    if isinstance(a, dict):
        assert a.keys() == b.keys()
        for k in a:
            _equal(a[k], b[k], f"{where}.{k}")
    elif isinstance(a, (tuple, list)):
        for i, (x, y) in enumerate(zip(a, b)):
            _equal(x, y, f"{where}[{i}]")
    else:
        assert torch.equal(torch.nan_to_num(a.double(), nan=-12345.0), torch.nan_to_num(b.double(), nan=-12345.0)), where


@pytest.mark.parametrize("name", ["activity_burst", "pump_score", "failed_spike", "top_gainer", "adx"])
def test_captured_pipeline_equals_eager(cuda, name):
    from binquant_amd import signals, strategies
    from binquant_amd.graphs import CapturedPipeline
    from binquant_amd.synth import device_panel

    fns = {
        "activity_burst": lambda o, h, l, c, v: strategies.activity_burst_features(o, h, l, c, v, v * c),
        "pump_score": lambda o, h, l, c, v: strategies.pump_score_features(o, h, l, c, v, c[0]),
        "failed_spike": lambda o, h, l, c, v: strategies.failed_spike_features(o, h, l, c, v, v * c),
        "top_gainer": lambda o, h, l, c, v: signals.top_gainer_features(o, h, l, c, v, v * c),
        "adx": lambda o, h, l, c, v: signals.adx(h, l, c),
    }
    fn = fns[name]
    a = device_panel(96, 400, seed=1)
    b = device_panel(96, 400, seed=2)
    ins_a = [a[k] for k in ("open", "high", "low", "close", "volume")]
    ins_b = [b[k] for k in ("open", "high", "low", "close", "volume")]
    g = CapturedPipeline(fn, *ins_a)
    _equal(g(*ins_a), fn(*ins_a), name)
    _equal(g(*ins_b), fn(*ins_b), name)
