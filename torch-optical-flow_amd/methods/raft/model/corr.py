"""``CorrBlock`` drop-in (reference: methods/raft/model/corr.py:37-87) on the gfx950 kernels.

* ``__init__`` — one launch of ``oflow_corr_pyramid_tiled_f32``: fp32 MFMA all-pairs volume with the 1/sqrt(C)
  scale and the floor 2x2 average-pool levels fused into the GEMM epilogue (`corr.py:38-54, 79-87`), stored in
  4x8 tiles (one 128-B line each) so that lookups touch about half the memory lines of row-major storage.
* ``__call__`` — one launch of ``oflow_corr_lookup_tiled_f32`` for all levels: the (2r+1)^2 bilinear window per
  level, written straight into the (B, L*(2r+1)^2, H, W) fp32 NCHW output (`corr.py:56-77`, `utils.py:64-80`).

Attributes match the reference: ``num_levels``, ``radius`` and ``corr_pyramid`` (list of (B*H*W, 1, H_l, W_l)
fp32 tensors), the latter rebuilt bit-exactly from the tiles on first access (after which lookups use it, so
in-place edits to it behave as in the reference). Divergence (documented): where a level is under 2 px in
H or W the reference returns NaN (it divides by W_l-1); this build raises ``ValueError`` at lookup time.
"""
from __future__ import annotations

import math
from typing import List, Optional

import torch
from torch import Tensor

from optical_flow import _native


class _CorrPyramidFn(torch.autograd.Function):
    """Training path: the pyramid (canonical levels) with a native backward -- level gradients folded through the
    average pools (oflow_corr_pyramid_grad_combine_f32), then grad_f1 = f2 . G^T / sqrt(C), grad_f2 = f1 . G / sqrt(C)
    as batched GEMMs (rocBLAS via torch.bmm)."""

    @staticmethod
    def forward(ctx, fmap1: Tensor, fmap2: Tensor, num_levels: int):
        ctx.save_for_backward(fmap1, fmap2)
        return tuple(_native.corr_pyramid(fmap1, fmap2, num_levels))

    @staticmethod
    def backward(ctx, *grads):
        f1, f2 = ctx.saved_tensors
        b, c, h, w = f1.shape
        n = h * w
        levels = [
            (g.contiguous().clone() if i == 0 else g.contiguous()) if g is not None else None for i, g in enumerate(grads)
        ]
        if levels[0] is None:
            levels[0] = torch.zeros((b * n, 1, h, w), device=f1.device, dtype=torch.float32)
        dims = _native.pyramid_dims(h, w, len(levels))
        levels = [g if g is not None else torch.zeros((b * n, 1, *d), device=f1.device) for g, d in zip(levels, dims)]
        g0 = _native.pyramid_grad_combine(levels).view(b, n, n)
        s = 1.0 / math.sqrt(c)
        f1m, f2m = f1.float().reshape(b, c, n), f2.float().reshape(b, c, n)
        g1 = torch.bmm(f2m, g0.transpose(1, 2)).mul_(s).view(b, c, h, w)
        g2 = torch.bmm(f1m, g0).mul_(s).view(b, c, h, w)
        return g1.to(f1.dtype), g2.to(f2.dtype), None


class _CorrLookupFn(torch.autograd.Function):
    """Training path: the windowed lookup over canonical levels with the native transpose
    (oflow_corr_lookup_backward_f32); coordinates get no gradient (the reference detaches them, raft.py:127)."""

    @staticmethod
    def forward(ctx, coords: Tensor, radius: int, *levels: Tensor):
        ctx.save_for_backward(coords)
        ctx.radius = radius
        ctx.shapes = [tuple(t.shape) for t in levels]
        ctx.device = coords.device
        return _native.corr_lookup(list(levels), coords, radius)

    @staticmethod
    def backward(ctx, grad_out):
        (coords,) = ctx.saved_tensors
        grads = [torch.zeros(sh, device=ctx.device, dtype=torch.float32) for sh in ctx.shapes]
        _native.corr_lookup_backward(grad_out.contiguous(), coords, ctx.radius, grads)
        return (None, None, *grads)


class CorrBlock:
    def __init__(self, fmap1: Tensor, fmap2: Tensor, num_levels: int = 4, radius: int = 4) -> None:
        self.num_levels = num_levels
        self.radius = radius
        self._pyramid: Optional[List[Tensor]] = None
        self._tiled = None
        self._batch = fmap1.shape[0]
        if torch.is_grad_enabled() and (fmap1.requires_grad or fmap2.requires_grad):
            # training (raft.py:149-175): canonical levels with native backward kernels
            self._pyramid = list(_CorrPyramidFn.apply(fmap1, fmap2, num_levels))
            self._grad = True
            return
        self._grad = False
        # lookups read the tiled layout (4x8 tiles = 128-B lines); the canonical list is built on first access
        self._tiled = _native.corr_pyramid_tiled(fmap1, fmap2, num_levels)

    @property
    def corr_pyramid(self) -> List[Tensor]:
        """The reference's ``corr_pyramid``: (B*H*W, 1, H_l, W_l) fp32 per level. Materialised on first access;
        from then on lookups read these tensors, so in-place edits behave as in the reference."""
        if self._pyramid is None:
            self._pyramid = [self._tiled.untile(l) for l in range(len(self._tiled.levels))]
            self._tiled = None
        return self._pyramid

    @corr_pyramid.setter
    def corr_pyramid(self, levels: List[Tensor]) -> None:
        self._pyramid = list(levels)
        self._tiled = None

    def __call__(self, coords: Tensor) -> Tensor:
        if self._tiled is not None:
            return _native.corr_lookup_tiled(self._tiled, coords, self.radius)
        if torch.is_grad_enabled() and any(t.requires_grad for t in self._pyramid):
            return _CorrLookupFn.apply(coords.detach(), self.radius, *self._pyramid)
        return _native.corr_lookup(self._pyramid, coords, self.radius)

    def lookup_nhwc(self, coords: Tensor, out: Tensor) -> Tensor:
        """The lookup as fp32 NHWC rows into ``out`` [B*H*W, L*(2r+1)^2] (an addition; the RAFT forward's convc1
        input): ``__call__(coords).permute(0, 2, 3, 1)`` written directly by the kernel, bit for bit."""
        if self._tiled is not None:
            return _native.corr_lookup_tiled_nhwc(self._tiled, coords, self.radius, out)
        b, _, h, w = coords.shape
        out.view(b, h, w, -1).copy_(_native.corr_lookup(self._pyramid, coords, self.radius).permute(0, 2, 3, 1))
        return out

    def batch_slice(self, b0: int, b1: int) -> "CorrBlock":
        """A CorrBlock over the pairs [b0, b1) sharing this one's levels (views, no copy): an addition, used by the RAFT
        forward to run pair halves on two streams."""
        view = CorrBlock.__new__(CorrBlock)
        view.num_levels, view.radius, view._grad = self.num_levels, self.radius, self._grad
        if self._tiled is not None:
            view._tiled, view._pyramid = self._tiled.batch_slice(b0, b1), None
        else:
            hw = self._pyramid[0].shape[0] // self._batch
            view._tiled, view._pyramid = None, [t[b0 * hw : b1 * hw] for t in self._pyramid]
        view._batch = b1 - b0
        return view

    @staticmethod
    def corr(fmap1: Tensor, fmap2: Tensor) -> Tensor:
        """All-pairs volume (B, H, W, 1, H, W) / sqrt(C) (`corr.py:79-87`)."""
        b, _, h, w = fmap1.shape
        return _native.corr_pyramid(fmap1, fmap2, 1)[0].view(b, h, w, 1, h, w)


class AlternateCorrBlock:
    """Memory-efficient correlation lookup (no (HW)^2 volume): same interface and output as ``CorrBlock``.

    Level-l correlations are computed on demand as dot products of fmap1 with the floor 2^l-pooled fmap2, which
    equals the dense pyramid by linearity of the pooling (`corr.py:38-54, 79-87`). Features are stored as NHWC
    fp16 and multiplied on v_mfma_f32_16x16x32_f16 with fp32 accumulation (BASELINE configs[4]: 1080p, fp16);
    outputs are fp32 like ``CorrBlock`` (Q5). Holds O(B*C*H*W) memory instead of O(B*(H*W)^2).
    """

    def __init__(self, fmap1: Tensor, fmap2: Tensor, num_levels: int = 4, radius: int = 4) -> None:
        self.num_levels = num_levels
        self.radius = radius
        self.fmap1_f16, self.fmap2_pyramid_f16 = _native.otf_prepare(fmap1, fmap2, num_levels)

    def __call__(self, coords: Tensor) -> Tensor:
        return _native.corr_lookup_otf(self.fmap1_f16, self.fmap2_pyramid_f16, coords, self.radius)

    def lookup_nhwc(self, coords: Tensor, out: Tensor) -> Tensor:
        """``__call__`` as fp32 NHWC rows [B*H*W, L*(2r+1)^2] into ``out`` (convc1's input)."""
        b, _, h, w = coords.shape
        out.view(b, h, w, -1).copy_(self(coords).permute(0, 2, 3, 1))
        return out
