"""Flow visualisation (drop-in for optical_flow/visualization/flow2rgb.py of the reference).

``flow2rgb`` keeps the reference's signature, argument meaning and errors (flow2rgb.py:19-73); the colour maps
(baker, hsv, meister: visualization/methods/*.py) run as two gfx950 kernels (csrc/flow_io.hip: per-image maxima,
then one fused colour pass) instead of ~25-40 ATen passes. Divergences: the field is computed in fp32 on the GPU
(a NumPy input is moved to the current ROCm device; a CPU tensor raises like every op of this build), NaN flow is
not supported (the reference indexes its colour wheel with garbage there), and ``max_norm`` must be >= 0.
"""
from __future__ import annotations

from pathlib import Path
from typing import Optional, Tuple, Union

import numpy as np
import torch
from torch import Tensor

from .. import _native

EPS = 1e-5
METHODS = [
    "baker",
    "hsv",
    "meister",
]


def flow2rgb(
    flow: Union[Tensor, np.ndarray],
    method: str = "baker",
    clip: Optional[Union[float, Tuple[float, float]]] = None,
    max_norm: Optional[float] = None,
    invert_y: bool = False,
) -> Tensor:
    """Flow (2, H, W) or (B, 2, H, W) -> RGB (3, H, W) or (B, 3, H, W) in [0, 1] (flow2rgb.py:19-73).

    ``clip`` clips the flow values (a scalar c means (-c, c)) before the normalisation by ``max_norm`` (default:
    each image's largest flow norm); ``invert_y`` negates the y component first. Raises ValueError for an unknown
    method, like the reference."""
    if method not in METHODS:
        raise ValueError(f"Unknown method: '{method}'.")
    if isinstance(flow, np.ndarray):
        flow = torch.as_tensor(flow, dtype=torch.float32, device=torch.device("cuda", torch.cuda.current_device()))
    ndims = flow.ndimension()
    if ndims == 3:
        flow = flow.unsqueeze(0)
    if clip is not None:
        clip = (-clip, clip) if not isinstance(clip, tuple) else clip
    denom = None
    if isinstance(max_norm, Tensor):
        if max_norm.numel() != 1:
            raise ValueError("flow2rgb: a tensor max_norm must hold one value")
        # tensor + EPS: the sum is rounded to fp32, like the reference's (max_norm + EPS)
        denom = float(max_norm.detach().float().cpu() + EPS)
    elif max_norm is not None:
        # Python float + EPS is a double sum; the division by it runs in fp32
        denom = float(np.float32(max_norm + EPS))
    # a colour map has no useful gradient: detach, so a prediction that requires grad (the reference's own
    # training_step logs flow2rgb(flow_predictions[-1]), raft.py:169-170) is visualised, not refused
    rgb = _native.flow2rgb(flow.detach(), method, clip, denom, invert_y)
    if ndims == 3:
        rgb = rgb.view(*rgb.shape[-3:])
    return rgb


def colorwheel(
    method: str = "baker",
    size: int = 256,
    file: Optional[Union[str, Path]] = None,
    device: Optional[torch.device] = None,
) -> Tensor:
    """Square (3, size, size) colour-wheel image of a visualisation method on a white background
    (flow2rgb.py:76-108); saved as PNG when ``file`` is given. Built on ``device`` (default: the current ROCm
    device) -- the reference builds it on the CPU."""
    device = device or torch.device("cuda", torch.cuda.current_device())
    h = w = size
    max_norm = size / 2
    dy, dx = torch.meshgrid(
        torch.linspace(-h / 2, h / 2, h, device=device), torch.linspace(-w / 2, w / 2, w, device=device),
        indexing="ij",
    )
    flow = torch.stack((dx, dy))
    norm = torch.norm(flow, dim=0, keepdim=True)
    rgb = flow2rgb(flow, method=method, max_norm=max_norm, invert_y=True)
    mask = torch.le(norm, max_norm)
    rgb = torch.where(mask, rgb, torch.ones_like(rgb))  # white background
    if file is not None:
        from PIL import Image

        rgb_numpy = rgb.mul(255).permute(1, 2, 0).type(torch.uint8).cpu().numpy()
        Image.fromarray(rgb_numpy, "RGB").save(file)
    return rgb
