"""Cross-symbol portfolio selectors.

The reference keeps, per cohort (the candle open_time for
LiquidationSweepPortfolioSelector, strategies/liquidation_sweep_pump.py:38-87;
the UTC hour for GradualGainerPortfolioSelector,
strategies/gradual_gainer_retest.py:33-70), the best candidate of each symbol
and dispatches the cohort's max (rank_score, symbol) once a later cohort
arrives; a candidate older than the latest cohort seen is rejected.

``select_winners`` does the whole decision for a batch of submissions on the
device: acceptance is a running maximum of the cohort key (torch.cummax),
the winner per cohort a segmented arg-max of (score, symbol, submission
order) with 64-bit atomics (bq_cohort_select) — the order the candidates of a
cohort arrive in does not change the winner, exactly as in the reference.
The two selector classes keep the reference's async API (submit / observe /
flush, same return values and dispatch order) and evaluate a cohort's winner
with the same kernel when it is dispatched.
"""

from __future__ import annotations

import ctypes
import logging
from collections.abc import Sequence
from dataclasses import dataclass

import numpy as np
import torch

from . import _lib, engine


@dataclass
class Winners:
    accepted: np.ndarray        # bool per submission (submit()'s return value)
    cohorts: np.ndarray         # int64 cohort keys, ascending = dispatch order
    winner: np.ndarray          # int64 submission index per cohort


def _device(device):
    if device is not None:
        return torch.device(device)
    if not torch.cuda.is_available():
        raise RuntimeError("portfolio selection needs a HIP device (no CPU fallback)")
    return torch.device("cuda")


def _cohort_winners(keys: torch.Tensor, sc: torch.Tensor, ranks: torch.Tensor, acc: torch.Tensor, stream=None):
    """Device segmented arg-max of (score, symbol rank, index) per cohort key
    over the accepted entries -> (sorted unique keys, winner index or -1)."""
    uniq, dense = torch.unique(keys, sorted=True, return_inverse=True)
    dense32 = dense.to(torch.int32).contiguous()
    acc8 = acc.to(torch.uint8).contiguous()
    sc = sc.contiguous()
    ranks = ranks.to(torch.int32).contiguous()
    nc = uniq.numel()
    scratch = torch.empty(2 * nc, dtype=torch.int64, device=keys.device)
    win = torch.empty(nc, dtype=torch.int64, device=keys.device)
    status = _lib.load().bq_cohort_select(
        keys.numel(), ctypes.c_void_p(dense32.data_ptr()), ctypes.c_void_p(acc8.data_ptr()),
        ctypes.c_void_p(sc.data_ptr()), ctypes.c_void_p(ranks.data_ptr()), nc, ctypes.c_void_p(scratch.data_ptr()),
        ctypes.c_void_p(win.data_ptr()), engine._stream_handle(stream))
    _lib.check(status, "bq_cohort_select")
    return uniq, win


def _accepted(keys: torch.Tensor) -> torch.Tensor:
    """submit() accepts a candidate unless its cohort is older than the latest seen."""
    run = torch.cummax(keys, 0).values
    prev = torch.cat([keys[:1], run[:-1]])
    return keys >= prev


def select_winners(cohort_keys, scores, symbols: Sequence[str], device=None, stream=None) -> Winners:
    """Submissions in arrival order -> accepted flags and each cohort's winner."""
    dev = _device(device)
    n = len(symbols)
    if n == 0:
        return Winners(np.zeros(0, bool), np.zeros(0, np.int64), np.zeros(0, np.int64))
    keys = torch.as_tensor(np.asarray(cohort_keys, dtype=np.int64)).to(dev)
    sc = torch.as_tensor(np.asarray(scores, dtype=np.float64)).to(dev)
    acc = _accepted(keys)
    # symbol strings -> ranks in Python's str order
    names = sorted(set(symbols))
    rank_of = {s: i for i, s in enumerate(names)}
    ranks = torch.tensor([rank_of[s] for s in symbols], dtype=torch.int32, device=dev)
    with engine.launch_scope(dev, stream, (keys, sc, ranks, acc)):
        uniq, win = _cohort_winners(keys, sc, ranks, acc)
    w = win.cpu().numpy()
    keep = w >= 0
    return Winners(acc.cpu().numpy(), uniq.cpu().numpy()[keep], w[keep])


def _all_gather_rows(rows: torch.Tensor, group) -> torch.Tensor:
    """all_gather of a variable number of int64 rows [n, k] -> [sum n, k]
    (counts first, then one padded gather; RCCL on device tensors, gloo
    through host memory)."""
    import torch.distributed as dist

    world = dist.get_world_size(group)
    on_host = dist.get_backend(group) == "gloo"
    xfer = rows.cpu() if on_host else rows
    n = torch.tensor([rows.shape[0]], dtype=torch.int64, device=xfer.device)
    counts = [torch.empty_like(n) for _ in range(world)]
    dist.all_gather(counts, n, group=group)
    counts = [int(c.item()) for c in counts]
    m = max(counts)
    pad = torch.zeros((m, rows.shape[1]), dtype=torch.int64, device=xfer.device)
    pad[:rows.shape[0]] = xfer
    parts = [torch.empty_like(pad) for _ in range(world)]
    dist.all_gather(parts, pad, group=group)
    out = torch.cat([p[:c] for p, c in zip(parts, counts)])
    return out.to(rows.device)


def select_winners_sharded(cohort_keys, scores, symbol_ids, seq, group=None, device=None, stream=None,
                           cohort_winners=None) -> Winners:
    """The portfolio decision when the symbols are sharded over ranks (SURVEY
    §8e): each rank holds the submissions of its own symbols; ``seq`` is the
    global arrival order and ``symbol_ids`` a global id in the symbols' str
    order (both shared by every rank, e.g. from the shard plan). Two
    exchanges: an all-gather of the (seq, key) pairs, from which each rank
    derives its submissions' acceptance (the running max of the key in
    arrival order), and an all-gather of each rank's per-cohort winners
    (key, score bits, symbol id, seq), merged by the same device arg-max.
    Every rank returns the same cohorts and winners (winner = global seq);
    ``accepted`` is per local submission. Equal to ``select_winners`` over
    the union of the submissions in seq order."""
    import torch.distributed as dist

    dev = _device(device)
    pick = cohort_winners or _cohort_winners
    # every launch and collective on `dev`, ordered per engine.launch_scope
    with engine.launch_scope(dev, stream):
        keys = torch.as_tensor(np.asarray(cohort_keys, dtype=np.int64)).to(dev)
        sc = torch.as_tensor(np.asarray(scores, dtype=np.float64)).to(dev)
        sid = torch.as_tensor(np.asarray(symbol_ids, dtype=np.int64)).to(dev)
        sq = torch.as_tensor(np.asarray(seq, dtype=np.int64)).to(dev)
        # (1) acceptance needs the global arrival order of the cohort keys
        pairs = _all_gather_rows(torch.stack([sq, keys], 1), group)
        order = torch.argsort(pairs[:, 0])
        gk = pairs[order, 1]
        excl = torch.cat([gk[:1], torch.cummax(gk, 0).values[:-1]])   # running max before each arrival
        pos = torch.searchsorted(pairs[order, 0].contiguous(), sq)
        acc = keys >= excl[pos] if keys.numel() else torch.zeros(0, dtype=torch.bool, device=dev)
        # (2) local winners per cohort (ties inside one symbol resolved by arrival order)
        local_order = torch.argsort(sq)
        k_l, s_l, i_l, q_l, a_l = keys[local_order], sc[local_order], sid[local_order], sq[local_order], acc[local_order]
        if k_l.numel():
            uniq, win = pick(k_l, s_l, i_l, a_l, None)
            ok = win >= 0
            w = win[ok]
            rows = torch.stack([uniq[ok], s_l[w].view(torch.int64), i_l[w], q_l[w]], 1)
        else:
            rows = torch.zeros((0, 4), dtype=torch.int64, device=dev)
        # (3) merge the ranks' winners: sorted by seq so that index order is arrival order
        allw = _all_gather_rows(rows, group)
        allw = allw[torch.argsort(allw[:, 3])]
        if allw.shape[0] == 0:
            return Winners(acc.cpu().numpy(), np.zeros(0, np.int64), np.zeros(0, np.int64))
        uniq, win = pick(allw[:, 0].contiguous(), allw[:, 1].contiguous().view(torch.float64), allw[:, 2].contiguous(),
                         torch.ones(allw.shape[0], dtype=torch.bool, device=dev), None)
        ok = win >= 0
        return Winners(acc.cpu().numpy(), uniq[ok].cpu().numpy(), allw[win[ok], 3].cpu().numpy())


class _CohortSelector:
    """Shared body of the two reference selectors (async API preserved)."""

    def __init__(self, device=None) -> None:
        self._latest: int | None = None
        self._candidates: dict[int, list] = {}
        self._device = device

    async def observe(self, candle_open_time: int) -> None:
        key = self._key_of_time(candle_open_time)
        if self._latest is not None and key <= self._latest:
            return
        for done in sorted(self._candidates):
            if done >= key:
                break
            await self._dispatch_winner(done)
        self._latest = key

    def _key_of_time(self, t: int) -> int:
        raise NotImplementedError

    async def submit(self, candidate) -> bool:
        await self.observe(candidate.candle_open_time)
        key = self._key_of_time(candidate.candle_open_time)
        if self._latest is not None and key < self._latest:
            return False
        self._candidates.setdefault(key, []).append(candidate)
        return True

    async def flush(self) -> None:
        for key in sorted(self._candidates):
            await self._dispatch_winner(key)

    async def _dispatch_winner(self, key: int) -> None:
        cohort = self._candidates.pop(key, [])
        if not cohort:
            return
        w = select_winners([key] * len(cohort), [c.rank_score for c in cohort], [c.symbol for c in cohort],
                           device=self._device)
        winner = cohort[int(w.winner[0])]
        try:
            await winner.dispatch()
        except Exception:
            logging.exception("%s portfolio winner failed for %s.", type(self).__name__, winner.symbol)


class LiquidationSweepPortfolioSelector(_CohortSelector):
    """One winner per candle cohort (strategies/liquidation_sweep_pump.py:38-87)."""

    def _key_of_time(self, t: int) -> int:
        return int(t)


class GradualGainerPortfolioSelector(_CohortSelector):
    """One winner per UTC hour (strategies/gradual_gainer_retest.py:33-70)."""

    def _key_of_time(self, t: int) -> int:
        return int(t) // 3_600_000
