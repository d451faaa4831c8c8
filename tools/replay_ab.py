"""Replay kernels A/B (LDS ring vs re-staged leaving values).
Run once per implementation: BQ_REPLAY_IMPL=ring|restage python tools/replay_ab.py
Prints one JSON line per (shape, case): mean ms and a digest of the outputs
(the two implementations must print identical digests)."""
import hashlib
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from binquant_amd import engine
from binquant_amd.engine import Ewm, Roll
from binquant_amd.synth import device_panel

impl = os.environ.get("BQ_REPLAY_IMPL", "auto") + os.environ.get("BQ_REPLAY_SPW", "")
for S, T, reps in ((1000, 400, 50), (12_500, 2_000, 10)):
    p = device_panel(S, T, seed=5)
    x = p["volume"].clone()
    x[:, 7::97] = float("nan")
    x[3, 100:160] = 1.0
    c = p["close"]
    cases = {
        "mean20": [Roll(x, 20, "mean")],
        "sum3_shift1": [Roll(x, 3, "sum", shift=1)],
        "std12": [Roll(c, 12, "std")],
        "var0_80": [Roll(c, 80, "var0" if "var0" in engine._lib.ROLL_MODES else "var", min_periods=5)],
        "ewm14": [Ewm(c, alpha=1 / 14, min_periods=14)],
        "batch8": [Roll(x, 20, "mean"), Roll(c, 12, "std"), Roll(c, 8, "std"), Roll(c, 20, "std"),
                   Roll(x, 2, "sum"), Roll(x, 3, "sum"), Roll(x, 5, "sum"), Roll(c, 10, "mean")],
        "batch16": [Roll(x, w, "mean") for w in (2, 5, 10, 20)] + [Roll(c, w, "std") for w in (8, 12, 20, 60)] +
                   [Roll(x, w, "sum") for w in (3, 6, 9, 12)] + [Ewm(c, span=s) for s in (9, 12, 20, 50)],
    }
    for name, specs in cases.items():
        outs = engine.rolling_many(*specs)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            outs = engine.rolling_many(*specs)
        e1.record()
        torch.cuda.synchronize()
        h = hashlib.sha1()
        for o in outs:
            h.update(o.cpu().numpy().tobytes())
        print(json.dumps({"impl": impl, "S": S, "T": T, "case": name, "ms": e0.elapsed_time(e1) / reps,
                          "digest": h.hexdigest()[:16]}), flush=True)
