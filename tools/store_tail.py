"""Tail of the live store tick (bench `store` leg shape: 10k symbols x 400-bar
histories): p50 / p99 / max over many ticks, the Python garbage collections
that fell inside timed ticks, and the same with the collector paused.
Usage: PYTHONPATH=. python tools/store_tail.py [ticks]"""
import gc
import sys
import time

import numpy as np
import torch

from binquant_amd.market_regime.store import DeviceLiveMarketContextAccumulator, DeviceMarketStateStore
from binquant_amd.synth import device_panel

N = int(sys.argv[1]) if len(sys.argv) > 1 else 1000
S, M = 10_000, 400
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
del hist, slots, tsh
vol = np.ones(S)
k = 0
in_tick = [False]
collections = []


def on_gc(phase, info):
    if phase == "start" and in_tick[0]:
        collections.append(info["generation"])


gc.callbacks.append(on_gc)


def run(n, label):
    global price, k
    lat = []
    collections.clear()
    for _ in range(n + 20):
        ts = t0 + 900_000 * (M + k)
        k += 1
        price = price * np.exp(rng.normal(0, 0.002, S))
        c = price
        torch.cuda.synchronize()
        in_tick[0] = True
        a = time.perf_counter()
        acc.on_closed_candles(syms, np.full(S, ts), c, c * 1.001, c * 0.999, c, vol, at=ts)
        torch.cuda.synchronize()
        b = time.perf_counter()
        in_tick[0] = False
        lat.append(b - a)
    lat = np.array(lat[20:]) * 1e3
    gens = {g: collections.count(g) for g in (0, 1, 2)}
    print(f"{label:14s} ticks {n}: p50 {np.percentile(lat, 50):.3f} p99 {np.percentile(lat, 99):.3f} "
          f"max {lat.max():.3f} ms; collections inside ticks by generation {gens}", flush=True)


run(N, "gc on")
gc.disable()
run(N, "gc disabled")
gc.enable()
gc.freeze()
run(N, "gc frozen")
run(N, "gc on (again)")
