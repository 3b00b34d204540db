"""Oracle: the ``optical_flow.operator`` functions on PyTorch-CPU. TEST INFRASTRUCTURE ONLY."""
from __future__ import annotations

from typing import Optional, Tuple, Union

import torch
import torch.nn.functional as F


def warp_grid(flow: torch.Tensor) -> torch.Tensor:
    """Base grid linspace(-1, 1) (x along W, y along H) + normalized flow (B, H, W, 2). `operator.py:36-56`."""
    b, h, w, _ = flow.shape
    gy, gx = torch.meshgrid(
        torch.linspace(-1.0, 1.0, h, device=flow.device), torch.linspace(-1.0, 1.0, w, device=flow.device), indexing="ij"
    )
    return torch.stack((gx, gy), dim=-1).unsqueeze(0).repeat(b, 1, 1, 1) + flow


def warp(frame, flow, mode: str = "bilinear", padding_mode: str = "border", align_corners: bool = False):
    """Inverse warp by grid_sample. `operator.py:8-33` (note Q8: not the identity at zero flow when
    align_corners=False, because the linspace base grid assumes align_corners=True)."""
    grid = warp_grid(flow.permute(0, 2, 3, 1))
    return F.grid_sample(frame, grid, mode=mode, padding_mode=padding_mode, align_corners=align_corners)


def scale(flow: torch.Tensor, factor: Union[float, Tuple[float, float]] = 1.0) -> torch.Tensor:
    """Per-component multiply (x by factor[0], y by factor[1]). `operator.py:59-82`."""
    assert flow.size(1) == 2
    if isinstance(factor, (float, int)):
        factor = (factor, factor)
    assert len(factor) == 2
    fx = torch.empty_like(flow[:, 0]).fill_(factor[0])
    fy = torch.empty_like(flow[:, 0]).fill_(factor[1])
    return flow * torch.stack((fx, fy), dim=1)


def resize(flow, size: Optional[Tuple[int, int]] = None, scale_factor: Optional[float] = None, mode: str = "bilinear"):
    """Spatial interpolate + magnitude rescale. `operator.py:85-114`."""
    assert flow.size(1) == 2
    assert flow.ndimension() == 4
    _, _, h, w = flow.shape
    if scale_factor:
        size = (round(h * scale_factor), round(w * scale_factor))
    resized = F.interpolate(flow, size, mode=mode)
    return scale(resized, (size[1] / w, size[0] / h))


def normalize(flow: torch.Tensor) -> torch.Tensor:
    """Pixel flow -> [-1, 1] grid units: x * 2/max(W-1,1), y * 2/max(H-1,1). `operator.py:117-130`."""
    assert flow.size(1) == 2
    h, w = flow.shape[-2:]
    return scale(flow, (2.0 / max(w - 1, 1), 2.0 / max(h - 1, 1)))


def denormalize(flow: torch.Tensor) -> torch.Tensor:
    """Inverse of ``normalize``. `operator.py:133-146`."""
    assert flow.size(1) == 2
    h, w = flow.shape[-2:]
    return scale(flow, (max(w - 1, 1) / 2, max(h - 1, 1) / 2))


def integrate(*flows: torch.Tensor) -> torch.Tensor:
    """total = f_k + warp(total, f_k) backwards over the sequence; the flow passed to ``warp`` is NOT
    normalized (Q9, `operator.py:149-165`)."""
    assert len(flows) >= 2
    total = flows[-1]
    for flow in reversed(flows[:-1]):
        assert flow.shape == total.shape, "All flows must have the same size."
        total = flow + warp(total, flow)
    return total
