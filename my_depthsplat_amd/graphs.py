"""hipGraph capture of a launch-bound render call (torch.cuda.CUDAGraph = hipGraph on ROCm).

The batched forward is host-sync-free whenever the worst-case key buffer fits
(raster.KEY_BUDGET_BYTES), so a whole decoder call — camera kernel, preprocess, scan,
scatter, per-tile sort, compositing — can be captured once and replayed with one launch,
removing the ~10 us host gaps between its kernels. Inputs must live in the tensors the
callable closes over (static buffers): copy new scenes into them before replay().
"""
from __future__ import annotations

import torch


class GraphedCall:
    """g = GraphedCall(lambda: decoder(gaussians, ...)); out = g() replays the captured work
    and returns the (static) outputs of the captured call."""

    def __init__(self, fn, warmup: int = 3):
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            for _ in range(warmup):  # also fills host-side caches (device index arrays)
                fn()
        torch.cuda.current_stream().wait_stream(side)
        torch.cuda.synchronize()
        self.graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(self.graph):
            self.out = fn()

    def __call__(self):
        self.graph.replay()
        return self.out
