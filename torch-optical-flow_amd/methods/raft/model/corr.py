"""``CorrBlock`` drop-in (reference: methods/raft/model/corr.py:37-87) on the gfx950 kernels.

* ``__init__`` — one launch of ``oflow_corr_pyramid_tiled_f32``: fp32 MFMA all-pairs volume with the 1/sqrt(C)
  scale and the floor 2x2 average-pool levels fused into the GEMM epilogue (`corr.py:38-54, 79-87`), stored in
  4x8 tiles (one 128-B line each) so that lookups touch about half the memory lines of row-major storage.
* ``__call__`` — one launch of ``oflow_corr_lookup_tiled_f32`` for all levels: the (2r+1)^2 bilinear window per
  level, written straight into the (B, L*(2r+1)^2, H, W) fp32 NCHW output (`corr.py:56-77`, `utils.py:64-80`).

Both are PyTorch operators (``torch.ops.oflow.corr_pyramid_tiled`` / ``corr_lookup_tiled``, csrc/torch_ops.cpp), so
``torch.compile(fullgraph=True)`` traces ``__call__`` without graph breaks; under autograd the canonical
``corr_pyramid`` / ``corr_lookup`` ops carry native backward formulas.

Attributes match the reference: ``num_levels``, ``radius`` and ``corr_pyramid`` (list of (B*H*W, 1, H_l, W_l)
fp32 tensors), the latter rebuilt bit-exactly from the tiles on first access (after which lookups use it, so
in-place edits to it behave as in the reference). Divergence (documented): where a level is under 2 px in
H or W the reference returns NaN (it divides by W_l-1); this build raises ``ValueError`` at lookup time.
"""
from __future__ import annotations

from typing import List, Optional

import torch
from torch import Tensor

from optical_flow import _native


class CorrBlock:
    def __init__(self, fmap1: Tensor, fmap2: Tensor, num_levels: int = 4, radius: int = 4) -> None:
        self.num_levels = num_levels
        self.radius = radius
        self._pyramid: Optional[List[Tensor]] = None
        self._tiled = None
        self._batch = fmap1.shape[0]
        if torch.is_grad_enabled() and (fmap1.requires_grad or fmap2.requires_grad):
            # training (raft.py:149-175): canonical levels; oflow::corr_pyramid / corr_lookup carry the native
            # backward (optical_flow/_ops.py)
            self._pyramid = _native.corr_pyramid(fmap1, fmap2, num_levels)
            self._grad = True
            return
        self._grad = False
        # lookups read the tiled layout (4x8 tiles = 128-B lines); the canonical list is built on first access
        self._tiled = _native.corr_pyramid_tiled(fmap1, fmap2, num_levels)

    @classmethod
    def from_split_features(cls, f1s: Tensor, f2s: Tensor, num_levels: int = 4, radius: int = 4) -> "CorrBlock":
        """A CorrBlock over feature maps given as S32 rows (B, H, W, C/32, 2, 32) -- the split-fp16 feature encoder's
        output -- with the pyramid built from split-fp16 products (oflow_corr_pyramid_tiled_s32): an addition, used
        by the RAFT forward (whose convolutions are split-fp16 already); values within the pyramid tolerance of the
        fp32 build. Inference only."""
        blk = cls.__new__(cls)
        blk.num_levels, blk.radius = num_levels, radius
        blk._pyramid, blk._grad, blk._batch = None, False, int(f1s.shape[0])
        blk._tiled = _native.corr_pyramid_tiled_s32(f1s, f2s, num_levels)
        return blk

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
