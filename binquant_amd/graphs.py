"""hipGraph capture of launch-bound pipelines (the live path).

On the live path the strategy pipelines run on frames of a few hundred bars
for a few hundred / thousand symbols per message: a pipeline
is 40-180 small launches (rolling batches, order statistics, element-wise
tails), so launch latency, not HBM, bounds it. ``CapturedPipeline`` records
one call into a hipGraph (torch.cuda.CUDAGraph drives hipStreamBeginCapture
on ROCm; every bq_* launch goes on torch's current stream, so it is captured
with the torch ops around it) and replays it with one submission. Inputs are
copied into the graph's static buffers; outputs are the graph's static
tensors (valid until the next replay).
"""

from __future__ import annotations

from collections.abc import Callable

import torch


class CapturedPipeline:
    def __init__(self, fn: Callable, *example_inputs: torch.Tensor, warmup: int = 2):
        if not torch.cuda.is_available():
            raise RuntimeError("CapturedPipeline needs a HIP device (no CPU fallback)")
        self.fn = fn
        self.static_in = [x.clone() for x in example_inputs]
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):   # warm-up: lazy allocations / attributes outside the capture
            for _ in range(warmup):
                fn(*self.static_in)
        torch.cuda.current_stream().wait_stream(side)
        torch.cuda.synchronize()
        self.graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(self.graph):
            self.static_out = fn(*self.static_in)

    def __call__(self, *inputs: torch.Tensor):
        if len(inputs) != len(self.static_in):
            raise ValueError(f"expected {len(self.static_in)} inputs, got {len(inputs)}")
        for dst, src in zip(self.static_in, inputs):
            if dst.shape != src.shape or dst.dtype != src.dtype:
                raise ValueError(f"input {tuple(src.shape)}/{src.dtype} does not match the captured "
                                 f"{tuple(dst.shape)}/{dst.dtype}")
            dst.copy_(src, non_blocking=True)
        self.graph.replay()
        return self.static_out
