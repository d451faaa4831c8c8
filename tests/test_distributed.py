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
        calls = []
        orig = dist.all_reduce

        def counting(*a, **k):
            calls.append(1)
            return orig(*a, **k)

        dist.all_reduce = counting
        try:
            part, n_total = reduce_partials(part, hi - lo)
        finally:
            dist.all_reduce = orig
        # one collective per context build, tracked count folded in
        assert len(calls) == 1 and n_total == S, (calls, n_total, S)
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


def _empty_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from binquant_amd.market_regime.batch import reduce_partials

        part, n = reduce_partials(torch.zeros((0, 10), dtype=torch.float64), 5 + rank)
        q.put((rank, n, tuple(part.shape)))
    finally:
        dist.destroy_process_group()


def test_reduce_partials_without_timestamps_agrees_on_total():
    """a [0, 10] partial (no timestamps) still yields the total
    tracked count over all ranks, the same on every rank."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_empty_worker, args=(r, 3, port, q)) for r in range(3)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert sorted(n for _, n, _ in res) == [18, 18, 18]
    assert all(shape == (0, 10) for _, _, shape in res)


def test_shard_bounds_cover_exactly():
    from binquant_amd.market_regime.batch import shard_bounds

    for S in (1, 7, 100, 12_500 * 8 + 3):
        for world in (1, 2, 3, 8):
            spans = [shard_bounds(S, world, r) for r in range(world)]
            assert spans[0][0] == 0 and spans[-1][1] == S
            assert all(a[1] == b[0] for a, b in zip(spans, spans[1:]))
            assert max(b - a for a, b in spans) - min(b - a for a, b in spans) <= 1


# ---- sharded portfolio selection (all-gather of per-cohort winners)

def _np_cohort_winners(keys, sc, ranks, acc, stream=None):
    """Stand-in for the device arg-max on CPU ranks: max (score, symbol, index)
    per cohort over the accepted entries (what bq_cohort_select computes)."""
    k, s, r, a = (t.numpy() for t in (keys, sc, ranks, acc))
    uniq = np.unique(k)
    win = np.full(len(uniq), -1, dtype=np.int64)
    for j, key in enumerate(uniq):
        idx = [i for i in range(len(k)) if k[i] == key and a[i]]
        if idx:
            win[j] = max(idx, key=lambda i: (s[i] + 0.0, r[i], i))
    return torch.from_numpy(uniq), torch.from_numpy(win)


def portfolio_shards(stream, world, rank, hourly):
    names = sorted({sym for _, sym, _ in stream})
    sid = {s: i for i, s in enumerate(names)}
    from binquant_amd.market_regime.batch import shard_bounds

    lo, hi = shard_bounds(len(names), world, rank)
    mine = [i for i, (_, sym, _) in enumerate(stream) if lo <= sid[sym] < hi]
    key = (lambda t: t // 3_600_000) if hourly else (lambda t: t)
    return (mine, [key(stream[i][0]) for i in mine], [stream[i][2] for i in mine],
            [sid[stream[i][1]] for i in mine])


def _portfolio_worker(rank, world, port, q, device):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from binquant_amd import portfolio

        runs = json.loads((G / "portfolio.json").read_text())
        pick = _np_cohort_winners if device == "cpu" else None
        out = []
        for name, rr in runs.items():
            for run in rr:
                stream = [tuple(x) for x in run["stream"]]
                mine, keys, scores, sids = portfolio_shards(stream, world, rank, name == "gradual")
                w = portfolio.select_winners_sharded(keys, scores, sids, mine, device=device, cohort_winners=pick)
                out.append((mine, w.accepted.tolist(), w.winner.tolist()))
        q.put((rank, out))
    finally:
        dist.destroy_process_group()


def run_sharded_portfolio(world, device):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_portfolio_worker, args=(r, world, port, q, device)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=300) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    runs = json.loads((G / "portfolio.json").read_text())
    want = [run for name in runs for run in runs[name]]
    for j, run in enumerate(want):
        acc = [None] * len(run["stream"])
        for r in range(world):
            mine, a, winners = res[r][j]
            assert winners == run["dispatched"], (r, j)   # every rank agrees on the winners
            for i, x in zip(mine, a):
                acc[i] = x
        assert acc == run["accepted"], j


@pytest.mark.parametrize("world", [2, 3])
def test_sharded_portfolio_selection_equals_reference(world):
    run_sharded_portfolio(world, "cpu")
