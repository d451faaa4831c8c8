"""Child process of tests/test_rolling_impls_gpu.py: runs a battery of
rolling / ewm / ffill series under the implementation forced by
BQ_RANK_IMPL / BQ_REPLAY_IMPL and saves the outputs (npz)."""
import sys

import numpy as np
import torch

from binquant_amd import engine
from binquant_amd.engine import Ewm, Ffill, Roll

RANK_JOBS = [(3, "max", 1.0, 1, 1), (6, "min", 0.0, 6, 1), (8, "quantile", 0.3, 4, 0), (12, "median", 0.5, 12, 0),
             (19, "median", 0.5, 19, 2), (24, "quantile", 0.75, 5, 0), (48, "quantile", 0.8, 48, 1),
             (65, "quantile", 0.92, 20, 1), (66, "median", 0.5, 1, 3), (80, "quantile", 0.92, 20, 1),
             (96, "quantile", 0.05, 30, 0), (60, "quantile", 0.85, 20, 1), (96, "qlower", 0.8, 20, 0),
             (96, "qlower", 0.8, 96, 2)]


def panel(S, T):
    g = torch.Generator().manual_seed(11)
    x = torch.randn(S, T, generator=g, dtype=torch.float64).cumsum(1)
    x[torch.rand(S, T, generator=g) < 0.03] = float("nan")
    x[1, 50:200] = 2.5                      # constant run
    x[2, :120] = float("nan")               # leading gap
    x[3, ::2] = -0.0
    x[4, 300:] = float("nan")               # trailing gap
    return x.cuda()


def main(out):
    S, T = 37, 700
    x = panel(S, T)
    res = {}
    rank = engine.rolling_many(*[Roll(x, w, st, q=q, min_periods=mp, shift=sh) for w, st, q, mp, sh in RANK_JOBS])
    for (w, st, q, mp, sh), r in zip(RANK_JOBS, rank):
        res[f"rank_{w}_{st}_{q}_{mp}_{sh}"] = r
    # rows shorter than two windows (one segment per row at the long windows)
    short = panel(6, 171)
    for (w, st, q, mp, sh), r in zip(RANK_JOBS, engine.rolling_many(
            *[Roll(short, w, st, q=q, min_periods=mp, shift=sh) for w, st, q, mp, sh in RANK_JOBS])):
        res[f"short_{w}_{st}_{q}_{mp}_{sh}"] = r
    # crossing flags beside plain quantiles (the flag instantiation of the
    # slide kernel where it runs, a flag pass after the other kernels)
    xj = [(48, 0.8, 48, 1), (80, 0.92, 20, 1), (60, 0.85, 20, 1), (19, 0.5, 19, 2)]
    thr, flags = engine.rolling_many(*[Roll(x, w, "quantile", q=q, min_periods=mp, shift=sh) for w, q, mp, sh in xj],
                                     cross=(0, 1, 3))
    for k, t in enumerate(thr):
        res[f"xthr_{k}"] = t
    for k, f in enumerate(flags):
        res[f"xflag_{k}"] = f
    mixed = [Roll(x, 2, "sum"), Roll(x, 12, "mean", shift=1), Roll(x, 20, "std"), Roll(x, 80, "var0", min_periods=5),
             Roll(x, 96, "std0", min_periods=1, shift=3), Ewm(x, alpha=1 / 14, min_periods=14), Ewm(x, span=50),
             Ffill(x)]
    for i, r in enumerate(engine.rolling_many(*mixed)):
        res[f"mixed_{i}"] = r
    for i, sp in enumerate(mixed):   # one class per call
        res[f"single_{i}"] = engine.rolling_many(sp)[0]
    big = panel(5000, 64)            # > 4096 symbols: the per-class path for a mixed batch
    for i, r in enumerate(engine.rolling_many(*[Roll(big, 3, "sum"), Roll(big, 10, "std"), Ewm(big, span=9)])):
        res[f"big_{i}"] = r
    np.savez(out, **{k: v.cpu().numpy() for k, v in res.items()})


if __name__ == "__main__":
    main(sys.argv[1])
