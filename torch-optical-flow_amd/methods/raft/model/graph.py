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

from optical_flow import _native

from . import update as _update

# A multi-pair forward is captured with its pair lanes (RAFT.pair_lanes) but without the per-lane side streams of the
# update block (update_block.split_streams): a side stream forked from a lane stream -- itself forked from the capture
# stream -- makes hipStreamEndCapture segfault inside the HIP runtime PyTorch bundles (torch/lib/libamdhip64.so, 7.0.x):
# the HIP-only reduction tools/exp/capture_fork_repro.hip crashes the same way on that runtime and captures correctly on
# ROCm 7.2's (profiles/r06/r6s10_*, r6s11_*). The same capture without those nested forks replays
# bit-identically, 18.57 ms vs 18.91 ms eager for 8 Sintel pairs (profiles/r05/s2_probe_noside.log). The model's
# settings are restored after the capture. None: capture as configured.
CAPTURE_LANE_SIDE_STREAMS = False

class GraphedRAFT:
    """``model(image0, image1, iters, test_mode=True)`` captured for the shapes of ``image0`` / ``image1``.

    Args:
        model: a ``RAFT`` on a ROCm device (eval or train mode as the caller wants; weights must not change after
            capture -- the packed-weight caches are built during the warm-up)
        image0, image1: (B, 3, H, W) example inputs (H, W divisible by 8: pad with ``InputPadder`` first)
        iters: GRU iterations
        warmup: eager forwards on a side stream before capture (allocator and weight caches settle)
        recorder: optional per-kernel timing recorder (``_native.set_event_recorder``; must hold ``"_native": True``),
            active during the capture only: its event pairs become event-record nodes of the graph, re-recorded by
            every replay, so after a replay they time that replay's launches (bench.py --graph)

    Calling the object with new images of the same shape returns ``(flow_low, flow_up)``: tensors owned by the graph,
    overwritten by the next call (clone them to keep them).
    """

    def __init__(self, model, image0: Tensor, image1: Tensor, iters: int = 12, warmup: int = 2, recorder=None) -> None:
        if recorder is not None and not recorder.get("_native"):
            raise ValueError("GraphedRAFT: a recorder needs native timing events ({'_native': True})")
        self.recorder = recorder
        if not image0.is_cuda:
            raise RuntimeError("GraphedRAFT: the inputs must be ROCm GPU tensors")
        self.model, self.iters = model, iters
        self.image0 = image0.detach().clone()
        self.image1 = image1.detach().clone()
        dev = image0.device
        blk = model.update_block
        side = getattr(blk, "split_streams", True)
        if CAPTURE_LANE_SIDE_STREAMS is not None and image0.shape[0] > 1 and getattr(model, "pair_lanes", 1) > 1:
            blk.split_streams = CAPTURE_LANE_SIDE_STREAMS
        try:
            self._capture(model, iters, warmup, dev)
        finally:
            blk.split_streams = side

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
            # capture_active(): the pair lanes' streams join the capture through event waits and on ROCm do not report
            # themselves as capturing; the weight caches must not wait on their (pre-capture) events from any of them
            prev = _native._recorder
            if self.recorder is not None:
                _native.set_event_recorder(self.recorder)
            try:
                with _update.capturing(dev), torch.cuda.graph(self.graph, stream=side):
                    self.flow_low, self.flow_up = model(self.image0, self.image1, iters=iters, test_mode=True)
            finally:
                if self.recorder is not None:
                    _native.set_event_recorder(prev)
            # the graph's event-record nodes point at these hipEvents: hold our own references, so that clearing or
            # replacing the caller's recorder dict cannot destroy an event a later replay still records into
            self._timing_events = [ev for k, v in (self.recorder or {}).items() if isinstance(v, list)
                                   for pair in v for ev in pair]

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
