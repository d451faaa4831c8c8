"""CPU oracle for binquant's indicator hot path — TEST INFRASTRUCTURE ONLY.

This package restates, in pandas/numpy, the reference algorithms the GPU path
replaces (every function cites the carkod/binquant file:line it follows). It is
imported ONLY by ``tests/``, ``__graft_entry__.smoke()`` and the
``cpu_baseline`` leg of ``bench.py`` — as the checker / CPU baseline, never as
the thing measured or shipped. ``binquant_amd`` never imports it and has no
CPU fallback.

Pinning (see DESIGN.md "Oracle"):
  * market_ref (live market context, regime annotation) and the strategy
    feature restatements are pinned against golden vectors produced by the
    real reference modules (tests/golden/make_golden.py imports
    /root/reference through a names-only shim in this container).
  * indicators_ref restates pybinbot.Indicators (pybinbot==1.11.8,
    uv.lock:1391-1403, a PyPI dependency absent from /root/reference and from
    this offline image). Its formulas are pinned only through the reference's
    in-repo formula twins (SMA-RSI bb_extreme_reversion.py:134-150,
    TR / EMA / BB live_market_context_accumulator.py:256-272) and the MFI
    bounds test (tests/test_coinrule_price_tracker.py:226-248); the remaining
    column formulas (macd_signal, twap, bb ddof, ATR smoothing) are
    **parity unpinned** against pybinbot itself.
"""
