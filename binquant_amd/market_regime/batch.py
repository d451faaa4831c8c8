"""Batched live-market-context over a [symbols x candles] panel.

Replaces, for every timestamp of the panel at once, the per-message loop of
LiveMarketContextAccumulator.refresh_context_for_timestamp
(market_regime/live_market_context_accumulator.py:72-84): the reference
recomputes _compute_symbol_features for every fresh symbol on every message
(O(S^2 * 400) per 15-minute period). Here:

  1. bq_market_features — per-symbol features at every t (device);
  2. bq_breadth_partial — per-t counts/sums over this rank's symbols (device,
     deterministic order);
  3. all_reduce(sum) of the [T x 10] partials over the symbol shards (RCCL
     over xGMI; the only collective of the whole hot path);
  4. scalar scoring + market-regime annotation over T (host, numpy).

BTC is replicated on every rank (one extra symbol), so relative strength and
the BTC regime score need no communication.
"""

from __future__ import annotations

from dataclasses import dataclass

import numpy as np
import torch
import torch.distributed as dist

from .. import engine
from .regime import ContextBatch, annotate_market, annotate_symbols, score_contexts


@dataclass
class MarketContextBatch:
    contexts: ContextBatch
    features: dict[str, torch.Tensor]   # this rank's [S, T] feature columns
    partial: torch.Tensor               # reduced [T, 10] partials (device)

    def context_at(self, i: int) -> dict | None:
        return self.contexts.context_at(i)

    def symbol_features_at(self, i: int, close: torch.Tensor, btc_return_t: float | None,
                           btc_index: int | None = None) -> dict[str, np.ndarray]:
        """Per-symbol feature row at timestamp index i (this rank's symbols),
        with relative strength and the micro-regime annotation. After a fused
        build (keep_features=False) only the last timestamp is held."""
        T = close.shape[1]
        j = i % T if i < 0 else i
        fcols = next(iter(self.features.values())).shape[1]
        if fcols == 1 and T > 1:
            if j != T - 1:
                raise ValueError("fused context build: only the last timestamp's features are kept")
            j_f = 0
        else:
            j_f = j
        f = {k: v[:, j_f].double().cpu().numpy() for k, v in self.features.items()}
        c = close[:, j].cpu().numpy()
        ret = f["return_pct"]
        rs = np.zeros_like(ret) if btc_return_t is None else ret - btc_return_t
        if btc_index is not None:
            rs[btc_index] = 0.0
        out = dict(f)
        out.update(close=c, above_ema20=c > f["ema20"], above_ema50=c > f["ema50"], relative_strength_vs_btc=rs)
        out.update(annotate_symbols(f["trend_score"], out["above_ema20"], out["above_ema50"], rs,
                                    f["bb_width"], f["atr_pct"], ret))
        return out


def shard_bounds(n_symbols: int, world: int, rank: int) -> tuple[int, int]:
    """Contiguous symbol block of `rank` (S/world per GPU)."""
    base, extra = divmod(n_symbols, world)
    lo = rank * base + min(rank, extra)
    return lo, lo + base + (1 if rank < extra else 0)


TRACKED_COLUMN = 9   # PARTIAL_COLUMNS[9]: symbols tracked by the shard


def reduce_partials(part: torch.Tensor, n_local: int, group=None, force: bool = False) -> tuple[torch.Tensor, int]:
    """ONE all_reduce(sum) of the [T, 10] partials over the symbol shards (RCCL
    over xGMI on GPUs, gloo on CPU). The shard's tracked-symbol
    count rides in the spare column 9 of every row, so the admission gate's
    total (live_market_context_accumulator.py:96-102) needs no second
    collective. Returns (reduced partials, total tracked symbols); on one
    rank the partials are returned with column 9 = n_local.

    force=True runs the collective whenever a process group is initialised,
    even at world size 1 (the one-GPU RCCL check, tests/test_rccl_gpu.py)."""
    part[:, TRACKED_COLUMN] = float(n_local)
    if dist.is_available() and dist.is_initialized() and (force or dist.get_world_size(group) > 1):
        # no timestamps (T == 0, the same on every rank): the count alone travels,
        # so every rank still agrees on the admission gate's total
        buf = part if part.shape[0] else torch.full((1, part.shape[1]), float(n_local), dtype=part.dtype,
                                                    device=part.device)
        if buf.is_cuda and dist.get_backend(group) == "gloo":   # CPU rehearsal of the RCCL path
            host = buf.cpu()
            dist.all_reduce(host, op=dist.ReduceOp.SUM, group=group)
            buf.copy_(host)
        else:   # RCCL over xGMI
            dist.all_reduce(buf, op=dist.ReduceOp.SUM, group=group)
        return part, int(buf[0, TRACKED_COLUMN].item())
    return part, int(n_local)


def contexts_from_partials(partial: np.ndarray, btc_return: np.ndarray, btc_trend: np.ndarray,
                           total_tracked: int, timestamps=None, previous_context: dict | None = None) -> ContextBatch:
    """Host scoring of reduced partials; btc_* are the benchmark's feature rows
    (NaN where it has no features)."""
    btc_valid = ~np.isnan(btc_return)
    batch = score_contexts(partial, np.nan_to_num(btc_return), np.nan_to_num(btc_trend), btc_valid,
                           total_tracked=total_tracked, timestamps=timestamps)
    return annotate_market(batch, previous_context)


def market_context_batch(
    high: torch.Tensor,
    low: torch.Tensor,
    close: torch.Tensor,
    btc_hlc: tuple[torch.Tensor, torch.Tensor, torch.Tensor],
    max_bars: int = 400,
    timestamps: np.ndarray | None = None,
    total_tracked: int | None = None,
    group=None,
    previous_context: dict | None = None,
    keep_features: bool = True,
) -> MarketContextBatch:
    """Contexts at every timestamp of a (possibly sharded) [S, T] panel.

    btc_hlc: the benchmark's (high, low, close) [1, T] rows, replicated.
    total_tracked: symbols tracked across ALL ranks (default: sum of shards).
    keep_features=False: the fused build (engine.context_partials) — the
    feature columns are never written; ``features`` then holds the last
    timestamp's row only ([S, 1] each: symbol_features_at(T - 1) works).
    """
    if keep_features:
        feats = engine.market_features(high, low, close, max_bars=max_bars)
        part = engine.breadth_partial(close, feats)
    else:
        part, last = engine.context_partials(high, low, close, max_bars=max_bars, last=True)
        feats = {k: v[:, None] for k, v in last.items()}
    part, n_total = reduce_partials(part, close.shape[0], group)
    bh, bl, bc = btc_hlc
    bf = engine.market_features(bh, bl, bc, max_bars=max_bars)
    batch = contexts_from_partials(
        part.cpu().numpy(),
        bf["return_pct"][0].cpu().numpy(),
        bf["trend_score"][0].cpu().numpy(),
        total_tracked=total_tracked if total_tracked is not None else n_total,
        timestamps=timestamps,
        previous_context=previous_context,
    )
    return MarketContextBatch(contexts=batch, features=feats, partial=part)
