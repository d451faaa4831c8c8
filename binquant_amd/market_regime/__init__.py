"""Market context (breadth / regime) on the GPU: per-symbol features and
cross-symbol partial sums on device, RCCL all-reduce across symbol shards,
O(T) scalar scoring on the host."""

from .batch import MarketContextBatch, market_context_batch  # noqa: F401
from .regime import annotate_market, annotate_symbols, score_contexts  # noqa: F401
