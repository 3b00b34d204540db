"""``optical_flow.operator`` drop-in (reference: optical_flow/operator/operator.py:8-165).

``warp`` runs on the gfx950 ``grid_warp`` kernel (the linspace base grid of ``warp_grid`` is fused into the
kernel, never materialised), registered as ``torch.ops.oflow.grid_warp`` with an autograd formula (frame and flow
gradients through ATen's grid_sampler_2d_backward on the same grid, optical_flow/_ops.py), so it traces under
torch.compile and differentiates in a photometric loss. The flow rescaling helpers are single elementwise passes and stay plain PyTorch
tensor ops, exactly as the reference writes them. Signatures, defaults, the asserts and
the quirks (Q8: ``warp`` is not the identity at zero flow with ``align_corners=False``; Q9: ``integrate`` passes
un-normalised flow to ``warp``) are the reference's.
"""
from __future__ import annotations

from typing import Optional, Tuple, Union

import torch
from torch import Tensor
from torch.nn import functional as F

from .. import _native


def warp(
    frame: Tensor,
    flow: Tensor,
    mode: str = "bilinear",
    padding_mode: str = "border",
    align_corners: bool = False,
) -> Tensor:
    """Inverse warping with optical flow (`operator.py:8-33`).

    Args:
        frame: the image tensor of shape (B, C, H, W), on a ROCm GPU
        flow: the optical flow tensor of shape (B, 2, H, W), already normalized (see :func:`normalize`)
        mode: 'bilinear' | 'nearest' | 'bicubic' (grid_sample semantics)
        padding_mode: 'zeros' | 'border' | 'reflection'
        align_corners: grid_sample's ``align_corners``

    Returns:
        The warped image (B, C, H, W) fp32.
    """
    return _native.grid_warp(frame, flow, mode, padding_mode, align_corners)


def warp_grid(flow: Tensor) -> Tensor:
    """Sampling grid (B, H, W, 2) = linspace(-1, 1) base grid + normalized flow (B, H, W, 2)
    (`operator.py:36-56`). ``warp`` does not call this: its kernel forms the same grid in registers."""
    b, h, w, _ = flow.shape
    range_x = torch.linspace(-1.0, 1.0, w, device=flow.device)
    range_y = torch.linspace(-1.0, 1.0, h, device=flow.device)
    grid_y, grid_x = torch.meshgrid(range_y, range_x, indexing="ij")
    grid = torch.stack((grid_x, grid_y), dim=-1).unsqueeze(0).repeat(b, 1, 1, 1)
    return grid + flow


def scale(flow: Tensor, factor: Union[float, Tuple[float, float]] = 1.0) -> Tensor:
    """Multiply the X component by factor[0] and Y by factor[1] (`operator.py:59-82`)."""
    assert flow.size(1) == 2
    if isinstance(factor, (float, int)):
        factor = (factor, factor)
    assert len(factor) == 2
    scale_w = torch.empty_like(flow[:, 0]).fill_(factor[0])
    scale_h = torch.empty_like(flow[:, 0]).fill_(factor[1])
    return flow * torch.stack((scale_w, scale_h), dim=1)


def resize(
    flow: Tensor,
    size: Optional[Tuple[int, int]] = None,
    scale_factor: Optional[float] = None,
    mode: str = "bilinear",
) -> Tensor:
    """Spatially resize a flow map and rescale its vectors accordingly (`operator.py:85-114`)."""
    assert flow.size(1) == 2
    assert flow.ndimension() == 4
    _, _, h, w = flow.shape
    if scale_factor:
        size = (round(h * scale_factor), round(w * scale_factor))
    sy = size[0] / h
    sx = size[1] / w
    resized = F.interpolate(flow, size, mode=mode)
    return scale(resized, (sx, sy))


def normalize(flow: Tensor) -> Tensor:
    """Pixel units -> [-1, 1] grid units (`operator.py:117-130`)."""
    assert flow.size(1) == 2
    h, w = flow.shape[-2:]
    return scale(flow, (2.0 / max(w - 1, 1), 2.0 / max(h - 1, 1)))


def denormalize(flow: Tensor) -> Tensor:
    """[-1, 1] grid units -> pixel units (`operator.py:133-146`)."""
    assert flow.size(1) == 2
    h, w = flow.shape[-2:]
    return scale(flow, (max(w - 1, 1) / 2, max(h - 1, 1) / 2))


def integrate(*flows: Tensor) -> Tensor:
    """Chain flows f_0..f_k into one map: total = f_i + warp(total, f_i) from the back (`operator.py:149-165`)."""
    assert len(flows) >= 2
    total = flows[-1]
    for flow in reversed(flows[:-1]):
        assert flow.shape == total.shape, "All flows must have the same size."
        total = flow + warp(total, flow)
    return total
