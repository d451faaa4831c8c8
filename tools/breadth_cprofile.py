"""cProfile of the C5 step (market_context_batch, keep_features=False) at the
bench's breadth shape: where the host time beyond the kernel goes.
Usage: python tools/breadth_cprofile.py [S T]"""
import cProfile
import pstats
import sys

import numpy as np
import torch

from binquant_amd.market_regime.batch import market_context_batch
from binquant_amd.synth import device_panel

S, T = (int(sys.argv[1]), int(sys.argv[2])) if len(sys.argv) > 2 else (100_000, 10_000)
p = device_panel(S, T, seed=1234)
h, l, c = p["high"], p["low"], p["close"]
btc = (h[:1], l[:1], c[:1])
tss = 1_700_000_000_000 + 900_000 * np.arange(T, dtype=np.int64)
for _ in range(2):
    market_context_batch(h, l, c, btc, timestamps=tss, keep_features=False)
torch.cuda.synchronize()
pr = cProfile.Profile()
pr.enable()
for _ in range(5):
    market_context_batch(h, l, c, btc, timestamps=tss, keep_features=False)
torch.cuda.synchronize()
pr.disable()
pstats.Stats(pr).sort_stats("cumulative").print_stats(30)
