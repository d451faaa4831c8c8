"""Does the output row pitch matter for the strategy passes as it did for
enrich at the shard (§2)? The activity-burst pass (bq_burst_features, 12.5k x
2k, 10 doubles + 8 byte columns per candle) timed with its outputs as [S, T]
views of [S, T + pad] buffers. Interleaved rounds; HIP-event time per launch.
Usage: PYTHONPATH=. python tools/strategy_pitch.py [pad ...]"""
import ctypes
import sys

import torch

from binquant_amd import _lib, engine, strategies
from binquant_amd.engine import BURST_BOOL_COLUMNS, BURST_FLOAT_COLUMNS, Roll as R
from binquant_amd.synth import device_panel

S, T = 12_500, 2_000
pads = [int(x) for x in sys.argv[1:]] or [0, 64, 192]
p = device_panel(S, T, seed=99)
o, h, l, c, v = (p[k] for k in ("open", "high", "low", "close", "volume"))
qv = v * c
bp = strategies.BurstParams()
bw = max(bp.lookback_window, 2)
med = engine.rolling_many(R(v, bw - 1, "median", min_periods=bw - 1, shift=2),
                          R(qv, bw - 1, "median", min_periods=bw - 1, shift=2))
ins = [o, h, l, c, v, qv, med[0], med[1]]
pr = _lib.BqBurstParams(float(bp.volume_multiplier), float(bp.quote_volume_multiplier), float(bp.price_threshold),
                        float(bp.min_baseline_volume), float(bp.min_range_frac), float(bp.min_body_frac),
                        float(bp.max_close_to_high), int(bp.min_recent_up_closes), 0)
lib = _lib.load()
res = {pad: [] for pad in pads}
for rnd in range(3):
    for pad in pads:
        ld = T + pad
        fo = [torch.empty((S, ld), dtype=torch.float64, device="cuda") for _ in BURST_FLOAT_COLUMNS]
        bo = [torch.empty((S, ld), dtype=torch.uint8, device="cuda") for _ in BURST_BOOL_COLUMNS]
        al = torch.empty((S, ld), dtype=torch.uint8, device="cuda")
        fp = _lib.ptr_array([t.data_ptr() for t in fo])
        bpp = _lib.ptr_array([t.data_ptr() for t in bo])
        ip = _lib.ptr_array([t.data_ptr() for t in ins])

        def f():
            _lib.check(lib.bq_burst_features(ip, S, T, T, ctypes.byref(pr), fp, bpp, ctypes.c_void_p(al.data_ptr()), ld,
                                             None), "bq_burst_features")

        for _ in range(2):
            f()
        torch.cuda.synchronize()
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
        ev[0].record()
        for _ in range(20):
            f()
        ev[1].record()
        torch.cuda.synchronize()
        res[pad].append(ev[0].elapsed_time(ev[1]) / 20)
        del fo, bo, al
for pad in pads:
    print(f"burst pass, pad {pad:4d}: {' '.join(f'{x:.4f}' for x in res[pad])} ms (best {min(res[pad]):.4f})", flush=True)
