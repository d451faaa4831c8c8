"""Multi-process (gloo, world_size 2, CPU) coverage of the sharded breadth path:
symbols split into contiguous blocks, per-shard [T, 10] partials, all_reduce,
host scoring — must equal the single-process contexts and the reference's
golden contexts. Partials come from the oracle here (no GPU on CPU ranks)."""

import json
import os
import socket
from pathlib import Path

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

G = Path(__file__).resolve().parent / "golden"


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _partials(h, l, c, idx, max_bars, lo, hi):
    from oracle import market_ref

    P = np.zeros((len(idx), 10))
    for j, t in enumerate(idx):
        for i in range(lo, hi):
            f = market_ref.panel_features_at(h[i], l[i], c[i], t, max_bars)
            if f is None:
                continue
            P[j] += [1, f["return_pct"] > 0, f["return_pct"] < 0, f["above_ema20"], f["above_ema50"],
                     f["return_pct"], f["trend_score"], f["atr_pct"], f["bb_width"], 0.0]
    return P


def _worker(rank, world, port, label, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from binquant_amd.market_regime.batch import contexts_from_partials, reduce_partials, shard_bounds
        from oracle import market_ref

        meta = json.loads((G / "market_context.json").read_text())
        panels = np.load(G / "market_context_panels.npz")
        sc = meta[label]
        ts_all = panels[f"{label}__timestamp"][0]
        h, l, c = (panels[f"{label}__{k}"] for k in ("high", "low", "close"))
        idx = [int(np.flatnonzero(ts_all == ts)[0]) for ts in sc["timestamps"]]
        S = c.shape[0]
        lo, hi = shard_bounds(S, world, rank)
        part = torch.from_numpy(_partials(h, l, c, idx, sc["max_bars"], lo, hi))
        part, n_total = reduce_partials(part, hi - lo)
        b = sc["symbols"].index(sc["btc"])   # BTC replicated on every rank
        btc = [market_ref.panel_features_at(h[b], l[b], c[b], t, sc["max_bars"]) for t in idx]
        ret = np.array([np.nan if f is None else f["return_pct"] for f in btc])
        trend = np.array([np.nan if f is None else f["trend_score"] for f in btc])
        batch = contexts_from_partials(part.numpy(), ret, trend, total_tracked=n_total,
                                       timestamps=np.array(sc["timestamps"]))
        if rank == 0:
            q.put([batch.context_at(i) for i in range(len(idx))])
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("label", ["random_64", "selloff_64"])
def test_two_rank_breadth_equals_reference(label):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, label, q)) for r in range(2)]
    for p in procs:
        p.start()
    got = q.get(timeout=300)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    meta = json.loads((G / "market_context.json").read_text())
    for g, want in zip(got, meta[label]["contexts"]):
        if want is None:
            assert g is None
            continue
        assert g["market_regime"] == want["market_regime"]
        assert g["advancers"] == want["advancers"] and g["decliners"] == want["decliners"]
        assert g["fresh_count"] == want["fresh_count"]
        for k in ("average_return", "average_relative_strength_vs_btc", "market_stress_score",
                  "long_tailwind", "short_tailwind", "average_atr_pct", "average_bb_width"):
            assert g[k] == pytest.approx(want[k], rel=1e-11, abs=1e-13), k


def test_shard_bounds_cover_exactly():
    from binquant_amd.market_regime.batch import shard_bounds

    for S in (1, 7, 100, 12_500 * 8 + 3):
        for world in (1, 2, 3, 8):
            spans = [shard_bounds(S, world, r) for r in range(world)]
            assert spans[0][0] == 0 and spans[-1][1] == S
            assert all(a[1] == b[0] for a, b in zip(spans, spans[1:]))
            assert max(b - a for a, b in spans) - min(b - a for a, b in spans) <= 1
