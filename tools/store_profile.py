"""cProfile of the live store tick at bench shape (10k symbols x 400-bar
histories): host cost of DeviceLiveMarketContextAccumulator.on_closed_candles.
Usage: python tools/store_profile.py [S]"""
import cProfile
import os
import pstats
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch

from binquant_amd.market_regime.store import DeviceLiveMarketContextAccumulator, DeviceMarketStateStore
from binquant_amd.synth import device_panel

S = int(sys.argv[1]) if len(sys.argv) > 1 else 10_000
M = 400
dev = torch.device("cuda")
syms = ["BTCUSDT"] + [f"S{i:05d}USDT" for i in range(1, S)]
store = DeviceMarketStateStore(max_bars_per_symbol=M, capacity=S)
acc = DeviceLiveMarketContextAccumulator(store, "BTCUSDT")
rng = np.random.default_rng(0)
price = 10 ** rng.uniform(-2, 3, S)
t0 = 1_700_000_000_000
hist = device_panel(S, M, device=dev, seed=5)
slots = torch.arange(S, dtype=torch.int64, device=dev).repeat_interleave(M)
for s in syms:
    store._slot(s)
tsh = (t0 + 900_000 * torch.arange(M, device=dev, dtype=torch.int64)).repeat(S)
store.update_slots(slots, tsh, [hist[k].reshape(-1) for k in ("open", "high", "low", "close", "volume")])
vol = np.ones(S)


def tick(k):
    global price
    ts = t0 + 900_000 * (M + k)
    price = price * np.exp(rng.normal(0, 0.002, S))
    c = price
    return acc.on_closed_candles(syms, np.full(S, ts), c, c * 1.001, c * 0.999, c, vol, at=ts)


for k in range(5):
    tick(k)
torch.cuda.synchronize()
lat = []
for k in range(5, 25):
    a = time.perf_counter()
    tick(k)
    torch.cuda.synchronize()
    lat.append(time.perf_counter() - a)
print(f"store tick p50 {np.percentile(np.array(lat) * 1e3, 50):.3f} ms")
pr = cProfile.Profile()
pr.enable()
for k in range(25, 45):
    tick(k)
torch.cuda.synchronize()
pr.disable()
pstats.Stats(pr).sort_stats("tottime").print_stats(30)
