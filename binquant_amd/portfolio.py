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


def select_winners(cohort_keys, scores, symbols: Sequence[str], device=None, stream=None) -> Winners:
    """Submissions in arrival order -> accepted flags and each cohort's winner."""
    dev = _device(device)
    n = len(symbols)
    keys = torch.as_tensor(np.asarray(cohort_keys, dtype=np.int64)).to(dev)
    sc = torch.as_tensor(np.asarray(scores, dtype=np.float64)).to(dev)
    if n == 0:
        return Winners(np.zeros(0, bool), np.zeros(0, np.int64), np.zeros(0, np.int64))
    # a submission is accepted unless its cohort is older than the latest seen
    run = torch.cummax(keys, 0).values
    prev = torch.cat([keys[:1], run[:-1]])
    acc = keys >= prev
    uniq, dense = torch.unique(keys, sorted=True, return_inverse=True)
    # symbol strings -> ranks in Python's str order
    names = sorted(set(symbols))
    rank_of = {s: i for i, s in enumerate(names)}
    ranks = torch.tensor([rank_of[s] for s in symbols], dtype=torch.int32, device=dev)
    dense32 = dense.to(torch.int32).contiguous()
    acc8 = acc.to(torch.uint8).contiguous()
    nc = uniq.numel()
    scratch = torch.empty(2 * nc, dtype=torch.int64, device=dev)
    win = torch.empty(nc, dtype=torch.int64, device=dev)
    status = _lib.load().bq_cohort_select(
        n, ctypes.c_void_p(dense32.data_ptr()), ctypes.c_void_p(acc8.data_ptr()), ctypes.c_void_p(sc.data_ptr()),
        ctypes.c_void_p(ranks.data_ptr()), nc, ctypes.c_void_p(scratch.data_ptr()), ctypes.c_void_p(win.data_ptr()),
        engine._stream_handle(stream))
    _lib.check(status, "bq_cohort_select")
    w = win.cpu().numpy()
    keep = w >= 0
    return Winners(acc.cpu().numpy(), uniq.cpu().numpy()[keep], w[keep])


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
