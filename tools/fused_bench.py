"""Cost of the fused element-wise interpreter (bq_fused_eval) per element-op:
programs of n chained ops over a [S, T] panel; prints ms and ns per
(element x op). Usage: python tools/fused_bench.py [S] [T]"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from binquant_amd import fused as F
from binquant_amd.synth import device_panel

S = int(sys.argv[1]) if len(sys.argv) > 1 else 12_500
T = int(sys.argv[2]) if len(sys.argv) > 2 else 2_000
p = device_panel(S, T, seed=1)
X, Y = F.inp(p["close"]), F.inp(p["volume"])
for n in (1, 8, 32, 96):
    e = X
    for k in range(n):
        e = (e * 1.0001 + Y) if k % 2 == 0 else (e - Y / 3.0)
    outs = {"y": e}
    P = F.build(list(outs.items()))
    F.run(outs)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    reps = 5
    e0.record()
    for _ in range(reps):
        F.run(outs)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / reps
    print(json.dumps({"ops_in_program": len(P.ins), "regs": P.n_regs, "ms": ms,
                      "ns_per_elem_op": ms * 1e6 / (S * T * len(P.ins)),
                      "GBps_io": S * T * 24 / ms / 1e6}), flush=True)
