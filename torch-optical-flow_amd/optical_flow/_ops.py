"""``torch.ops.oflow``: the correlation / warp path as PyTorch operators (csrc/torch_ops.cpp -> liboflow_torch.so).

The library registers, per op, a HIP-key kernel that calls the C ABI of liboflow_hip.so on PyTorch's current stream
and a Meta kernel (output shapes only, what torch.compile's fake-tensor tracing runs). This module loads it and
registers the autograd formulas on top, so ``CorrBlock`` and ``optical_flow.warp`` are ordinary traceable ops:
``torch.compile(fullgraph=True)`` captures them without graph breaks, and training differentiates through them.

Autograd:
  * ``corr_pyramid``: the level gradients go back through the floor 2x2 pools (native kernel) and two batched GEMMs
    (``corr_pyramid_backward``, fp32 MFMA): grad_f1 = f2 . G^T / sqrt(C), grad_f2 = f1 . G / sqrt(C).
  * ``corr_lookup``: the native transpose of the bilinear window gather (``corr_lookup_backward``); coords get no
    gradient -- the reference detaches them before every lookup (methods/raft/model/raft.py:127).
  * ``grid_warp`` / ``grid_sample``: the native transpose (``grid_warp_backward`` / ``grid_sample_backward``,
    csrc/warp_backward.hip: ATen grid_sampler_2d_backward's formulas, tap gradients added with fp32 atomics); the
    warp's base grid is constant, so the flow gradient is the grid gradient.
The tiled / NHWC / fp16 on-the-fly lookups are the inference layouts and have no autograd formula.
"""
from __future__ import annotations

import os

import torch

_OPS_PATH = os.environ.get(
    "OFLOW_OPS_LIB", os.path.join(os.path.dirname(os.path.abspath(__file__)), "_lib", "liboflow_torch.so")
)
OPS = (
    "corr_pyramid",
    "corr_pyramid_tiled",
    "corr_lookup",
    "corr_lookup_tiled",
    "corr_lookup_tiled_nhwc",
    "corr_otf_prepare",
    "corr_lookup_otf",
    "grid_warp",
    "grid_sample",
    "corr_lookup_backward",
    "corr_pyramid_backward",
    "grid_warp_backward",
    "grid_sample_backward",
)
_loaded = False


def library_path() -> str:
    return _OPS_PATH


def load() -> None:
    """Load liboflow_torch.so once and register the autograd formulas. Raises RuntimeError if it is missing."""
    global _loaded
    if _loaded:
        return
    if not os.path.exists(_OPS_PATH):
        raise RuntimeError(
            f"liboflow_torch.so not found at {_OPS_PATH}: build it with `make -C torch-optical-flow_amd/csrc` "
            "(or __graft_entry__.build()); the MI355X path has no CPU fallback"
        )
    torch.ops.load_library(_OPS_PATH)
    _register_autograd()
    _loaded = True


# ---------------------------------------------------------------------------------------------- autograd formulas
def _pyramid_setup(ctx, inputs, output):
    fmap1, fmap2, _ = inputs
    ctx.save_for_backward(fmap1, fmap2)
    ctx.shapes = [tuple(t.shape) for t in output]


def _pyramid_backward(ctx, grads):
    fmap1, fmap2 = ctx.saved_tensors
    levels = [
        g.contiguous() if g is not None else torch.zeros(sh, device=fmap1.device, dtype=torch.float32)
        for g, sh in zip(grads, ctx.shapes)
    ]
    g1, g2 = torch.ops.oflow.corr_pyramid_backward(levels, fmap1, fmap2)
    return g1, g2, None


def _lookup_setup(ctx, inputs, output):
    levels, coords, radius = inputs
    # the native transpose rebuilds every level's size from level 0 by floor 2x2 pooling (corr.py:53): levels of any
    # other size are refused here, in the forward, instead of failing with a gradient-shape error in the backward
    h, w = (int(v) for v in levels[0].shape[-2:])
    for lv in levels:
        if tuple(int(v) for v in lv.shape[-2:]) != (h, w):
            raise RuntimeError(
                f"corr_lookup backward: level sizes must be the floor 2x2 pools of level 0 (expected {(h, w)}, got "
                f"{tuple(lv.shape[-2:])})")
        h, w = h // 2, w // 2
    ctx.save_for_backward(coords)
    ctx.radius = radius
    ctx.level0 = tuple(levels[0].shape[-2:])
    ctx.nl = len(levels)


def _lookup_backward(ctx, grad_out):
    (coords,) = ctx.saved_tensors
    h0, w0 = ctx.level0
    grads = torch.ops.oflow.corr_lookup_backward(grad_out.contiguous(), coords, ctx.radius, h0, w0, ctx.nl)
    return list(grads), None, None


def _warp_setup(ctx, inputs, output):
    frame, flow, mode, pad, ac = inputs
    ctx.save_for_backward(frame, flow)
    ctx.args = (mode, pad, ac)


def _warp_backward(ctx, grad_out):
    frame, flow = ctx.saved_tensors
    mode, pad, ac = ctx.args
    # the native transpose (warp_backward.hip): grid = linspace base + flow, so the flow gradient is the grid gradient
    # only the wanted outputs are formed (no zero fill / atomics for a frame that needs no gradient)
    need = [bool(ctx.needs_input_grad[0]), bool(ctx.needs_input_grad[1])]
    g_in, g_flow = torch.ops.oflow.grid_warp_backward(grad_out.contiguous(), frame, flow, mode, pad, ac, need)
    g_frame = g_in.to(frame.dtype) if need[0] else None
    g_flow = g_flow.to(flow.dtype) if need[1] else None
    return g_frame, g_flow, None, None, None


def _sample_setup(ctx, inputs, output):
    inp, grid, mode, pad, ac = inputs
    ctx.save_for_backward(inp, grid)
    ctx.args = (mode, pad, ac)


def _sample_backward(ctx, grad_out):
    inp, grid = ctx.saved_tensors
    mode, pad, ac = ctx.args
    need = [bool(ctx.needs_input_grad[0]), bool(ctx.needs_input_grad[1])]
    g_in, g_grid = torch.ops.oflow.grid_sample_backward(grad_out.contiguous(), inp, grid, mode, pad, ac, need)
    g_x = g_in.to(inp.dtype) if need[0] else None
    g_g = g_grid.to(grid.dtype) if need[1] else None
    return g_x, g_g, None, None, None


def _register_autograd() -> None:
    reg = torch.library.register_autograd
    reg("oflow::corr_pyramid", _pyramid_backward, setup_context=_pyramid_setup)
    reg("oflow::corr_lookup", _lookup_backward, setup_context=_lookup_setup)
    reg("oflow::grid_warp", _warp_backward, setup_context=_warp_setup)
    reg("oflow::grid_sample", _sample_backward, setup_context=_sample_setup)
