"""The breadth reduction's RCCL branch on hardware (the one
collective of the hot path; reference: the per-message reduction of
market_regime/live_market_context_accumulator.py:95-163).

A one-GPU box cannot form a multi-rank RCCL ring, so a world-size-1 "nccl"
process group drives reduce_partials(force=True) through dist.all_reduce on
the device buffer — RCCL's own launch path — and the result must equal, bit
for bit, the same partials reduced through a gloo group (the CPU rehearsal the
multi-rank tests use) and the unreduced partials (a sum over one rank). The
scored contexts built from either reduction are equal. Runs in a child
process so the process group does not outlive the test."""

import os
import socket
import subprocess
import sys
import textwrap

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

SCRIPT = textwrap.dedent("""
    import os, sys
    import numpy as np
    import torch
    import torch.distributed as dist
    sys.path.insert(0, {root!r})
    from binquant_amd import engine
    from binquant_amd.market_regime.batch import reduce_partials, contexts_from_partials
    from binquant_amd.synth import device_panel

    torch.cuda.set_device(0)
    dist.init_process_group("nccl", device_id=torch.device("cuda", 0), rank=0, world_size=1,
                            init_method="tcp://127.0.0.1:{port}")
    assert dist.get_backend() == "nccl"
    gloo = dist.new_group(backend="gloo")
    calls = []
    real = dist.all_reduce

    def spy(t, *a, **k):
        calls.append((t.device.type, dist.get_backend(k.get("group"))))
        return real(t, *a, **k)

    dist.all_reduce = spy
    S, T = 3000, 1200
    p = device_panel(S, T, seed=11)
    part, _ = engine.context_partials(p["high"], p["low"], p["close"], max_bars=400)
    base = part.clone()
    base[:, 9] = float(S)
    a, na = reduce_partials(part.clone(), S, force=True)               # RCCL, device buffer
    b, nb = reduce_partials(part.clone(), S, group=gloo, force=True)   # gloo, host copy
    torch.cuda.synchronize()
    assert calls == [("cuda", "nccl"), ("cpu", "gloo")], calls
    assert na == nb == S, (na, nb)
    assert torch.equal(a, b), "RCCL and gloo reductions differ"
    assert torch.equal(a, base), "a one-rank sum must return the partials"
    # a second RCCL reduction on a fresh buffer (the per-step call of the bench)
    c, nc = reduce_partials(part.clone(), S, force=True)
    assert torch.equal(c, a) and nc == S
    z = np.zeros(T)
    ca = contexts_from_partials(a.cpu().numpy(), z, z, total_tracked=na)
    cb = contexts_from_partials(b.cpu().numpy(), z, z, total_tracked=nb)
    assert (ca.valid == cb.valid).all() and ca.valid.any()
    for k, v in ca.fields.items():
        w = cb.fields[k]
        assert (np.array_equal(v, w, equal_nan=True) if v.dtype.kind == "f" else (v == w).all()), k
    dist.destroy_process_group()
    print("RCCL_OK", len(calls))
""")


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_reduce_partials_rccl_world1_equals_gloo(cuda):
    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    r = subprocess.run([sys.executable, "-c", SCRIPT.format(root=ROOT, port=_free_port())], env=env,
                       capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    assert "RCCL_OK 3" in r.stdout
