"""Where the C5 step's time goes beyond the context kernel (bench.py breadth
leg shape, one GPU): the kernel launch, the partials' reduction, the
benchmark's feature row, the D2H copies and the host scoring, each timed
synchronously over a few steps. Usage: python tools/breadth_parts.py [S T]"""
import sys
import time

import numpy as np
import torch

from binquant_amd import engine
from binquant_amd.market_regime.batch import contexts_from_partials, market_context_batch, reduce_partials
from binquant_amd.synth import device_panel

S, T = (int(sys.argv[1]), int(sys.argv[2])) if len(sys.argv) > 2 else (100_000, 10_000)
p = device_panel(S, T, seed=1234)
h, l, c = p["high"], p["low"], p["close"]
btc = (h[:1], l[:1], c[:1])
tss = 1_700_000_000_000 + 900_000 * np.arange(T, dtype=np.int64)


def t(fn, n=5):
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n):
        r = fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / n * 1e3, r


ms_all, _ = t(lambda: market_context_batch(h, l, c, btc, timestamps=tss, keep_features=False))
ms_k, (part, last) = t(lambda: engine.context_partials(h, l, c, max_bars=400, last=True))
ms_red, (pr, n_total) = t(lambda: reduce_partials(part, S))
ms_bf, bf = t(lambda: engine.market_features(*btc, max_bars=400))
ms_d2h, ph = t(lambda: (pr.cpu().numpy(), bf["return_pct"][0].cpu().numpy(), bf["trend_score"][0].cpu().numpy()))
ms_sc, _ = t(lambda: contexts_from_partials(ph[0], ph[1], ph[2], total_tracked=n_total, timestamps=tss))
print(f"step {ms_all:.3f} ms = kernel(+last) {ms_k:.3f} + reduce {ms_red:.3f} + bench features {ms_bf:.3f} "
      f"+ D2H {ms_d2h:.3f} + scoring {ms_sc:.3f} (sum {ms_k + ms_red + ms_bf + ms_d2h + ms_sc:.3f})")
