"""RAFT inference replayed from a HIP graph (an addition for fixed-shape serving; not in the reference).

At batch 1 the test-mode forward of ``RAFT`` (methods/raft/model/raft.py:87-147, driven per pair by
methods/raft/predict.py:73-89) issues ~30 short kernels per GRU iteration; from Python each launch costs several
microseconds of host time, which at 1/8 resolution is comparable to the kernels themselves. ``GraphedRAFT``
captures the whole forward -- encoders on their side stream, the correlation pyramid, every update iteration and
the convex upsampling -- once per (batch, H, W, iters) into a ``torch.cuda.CUDAGraph`` (a hipGraph on ROCm) and
replays it: one launch per pair batch, inputs copied into the captured buffers first.

The replayed forward is the same kernel sequence as the eager one, so the flows are bit-identical to
``model(image0, image1, iters=iters, test_mode=True)`` (tests/test_gpu_raft.py checks it).
"""
from __future__ import annotations

from typing import Tuple

import torch
from torch import Tensor


class GraphedRAFT:
    """``model(image0, image1, iters, test_mode=True)`` captured for the shapes of ``image0`` / ``image1``.

    Args:
        model: a ``RAFT`` on a ROCm device (eval or train mode as the caller wants; weights must not change after
            capture -- the packed-weight caches are built during the warm-up)
        image0, image1: (B, 3, H, W) example inputs (H, W divisible by 8: pad with ``InputPadder`` first)
        iters: GRU iterations
        warmup: eager forwards on a side stream before capture (allocator and weight caches settle)

    Calling the object with new images of the same shape returns ``(flow_low, flow_up)``: tensors owned by the graph,
    overwritten by the next call (clone them to keep them).
    """

    def __init__(self, model, image0: Tensor, image1: Tensor, iters: int = 12, warmup: int = 2) -> None:
        if not image0.is_cuda:
            raise RuntimeError("GraphedRAFT: the inputs must be ROCm GPU tensors")
        self.model, self.iters = model, iters
        self.image0 = image0.detach().clone()
        self.image1 = image1.detach().clone()
        dev = image0.device
        # multi-pair batches are captured with one pair lane: capturing the two-lane update loop (each lane with its
        # own side stream) segfaults inside capture_end (profiles/r04/s12_graph8.log); one lane captures and replays
        # bit-identically to the eager forward (tools/exp/graph_probe.py, 8 pairs: replay 19.72 ms vs eager two-lane
        # 19.62 ms, profiles/r04/s32_graph8l1.log). The model's own setting is restored after the capture.
        lanes = getattr(model, "pair_lanes", 1)
        if image0.shape[0] > 1 and lanes > 1:
            model.pair_lanes = 1
        try:
            self._capture(model, iters, warmup, dev)
        finally:
            model.pair_lanes = lanes

    def _capture(self, model, iters: int, warmup: int, dev) -> None:
        with torch.inference_mode():
            side = torch.cuda.Stream(device=dev)
            side.wait_stream(torch.cuda.current_stream(dev))
            with torch.cuda.stream(side):
                for _ in range(max(1, warmup)):
                    model(self.image0, self.image1, iters=iters, test_mode=True)
            torch.cuda.current_stream(dev).wait_stream(side)
            torch.cuda.synchronize(dev)
            self.graph = torch.cuda.CUDAGraph()
            # captured on the warm-up stream: the side / lane streams the forward forks to (keyed by their owner
            # stream, model/update.py _side_stream) are the ones the warm-up created
            with torch.cuda.graph(self.graph, stream=side):
                self.flow_low, self.flow_up = model(self.image0, self.image1, iters=iters, test_mode=True)

    def __call__(self, image0: Tensor, image1: Tensor) -> Tuple[Tensor, Tensor]:
        if image0.shape != self.image0.shape or image1.shape != self.image1.shape:
            raise ValueError(
                f"GraphedRAFT: captured for {tuple(self.image0.shape)}, got {tuple(image0.shape)} / {tuple(image1.shape)}"
            )
        self.image0.copy_(image0, non_blocking=True)
        self.image1.copy_(image1, non_blocking=True)
        guard = getattr(self.model, "range_guard", "off") in ("sync", "deferred")
        if guard:  # (the captured forward cannot read the range flag: the model's guard runs around the replay)
            self.model._range_before(self.image0.device)
        self.graph.replay()
        if guard:
            self.model._range_after(self.image0.device)
        return self.flow_low, self.flow_up
