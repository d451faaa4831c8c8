"""binquant_amd — MI355X (gfx950) engine for binquant's technical-indicator hot path.

Layers:
  * ``include/binquant_amd.h`` — the C ABI (device pointers, int status);
  * ``binquant_amd._lib``      — ctypes binding of the in-tree HIP library;
  * ``binquant_amd.engine``    — batched [S, T] device entry points;
  * ``binquant_amd.indicators``— pybinbot.Indicators-compatible DataFrame API;
  * ``binquant_amd.market_regime`` — accumulator / state-store mirrors.
There is no CPU fallback anywhere: a missing library raises.
"""

__version__ = "0.1.0"
