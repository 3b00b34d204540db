"""``model.utils`` drop-in (reference: methods/raft/model/utils.py:38-91)."""
from __future__ import annotations

from typing import List, Optional, Sequence, Tuple, Union

import torch
import torch.nn.functional as F
from torch import Tensor

from optical_flow import _native


class InputPadder:
    """Pads images such that dimensions are divisible by 8 (`utils.py:38-61`): replicate padding, symmetric in
    'sintel' mode, left/right + bottom only in every other mode (Q10)."""

    def __init__(self, dims: Sequence[int], mode: str = "sintel") -> None:
        self.ht, self.wd = dims[-2:]
        pad_ht = (((self.ht // 8) + 1) * 8 - self.ht) % 8
        pad_wd = (((self.wd // 8) + 1) * 8 - self.wd) % 8
        if mode == "sintel":
            self._pad = [pad_wd // 2, pad_wd - pad_wd // 2, pad_ht // 2, pad_ht - pad_ht // 2]
        else:
            self._pad = [pad_wd // 2, pad_wd - pad_wd // 2, 0, pad_ht]

    def pad(self, *inputs: Tensor) -> List[Tensor]:
        # GPU fp32 frames (the inference inputs): every frame in one native launch (oflow_replicate_pad_f32, a copy,
        # bit-exact); anything else (CPU, autograd, other dtypes) through F.pad as the reference
        if (1 <= len(inputs) <= 4 and all(isinstance(x, Tensor) and x.is_cuda and x.dtype == torch.float32
                                          and x.dim() >= 2 and x.shape == inputs[0].shape for x in inputs)
                and not (torch.is_grad_enabled() and any(x.requires_grad for x in inputs))):
            return _native.replicate_pad(inputs, self._pad)
        return [F.pad(x, self._pad, mode="replicate") for x in inputs]

    def unpad(self, x: Tensor) -> Tensor:
        ht, wd = x.shape[-2:]
        c = [self._pad[2], ht - self._pad[3], self._pad[0], wd - self._pad[1]]
        return x[..., c[0] : c[1], c[2] : c[3]]


def bilinear_sampler(
    img: Tensor, coords: Tensor, mode: str = "bilinear", mask: bool = False
) -> Union[Tensor, Tuple[Tensor, Tensor]]:
    """grid_sample with pixel coordinates, align_corners=True, zeros padding (`utils.py:64-80`); like the
    reference it ignores ``mode``. Sampling runs on the gfx950 ``grid_sample`` kernel."""
    h, w = img.shape[-2:]
    xgrid, ygrid = coords.split([1, 1], dim=-1)
    xgrid = 2 * xgrid / (w - 1) - 1
    ygrid = 2 * ygrid / (h - 1) - 1
    grid = torch.cat([xgrid, ygrid], dim=-1)
    out = _native.grid_sample(img, grid, "bilinear", "zeros", True)
    if mask:
        m = (xgrid > -1) & (ygrid > -1) & (xgrid < 1) & (ygrid < 1)
        return out, m.float()
    return out


def coords_grid(batch: int, ht: int, wd: int, device: Optional[torch.device] = None) -> Tensor:
    """(B, 2, ht, wd) fp32, channel 0 = x (column index), channel 1 = y (row index) (`utils.py:83-86`).
    ``device`` (an addition) builds it in place instead of on the CPU + copy (`raft.py:68-69`)."""
    ys, xs = torch.meshgrid(
        torch.arange(ht, device=device, dtype=torch.float32),
        torch.arange(wd, device=device, dtype=torch.float32),
        indexing="ij",
    )
    return torch.stack((xs, ys), dim=0)[None].repeat(batch, 1, 1, 1)


def upflow8(flow: Tensor, mode: str = "bilinear") -> Tensor:
    """8x bilinear upsampling of a flow field, magnitudes x8 (`utils.py:89-91`)."""
    new_size = (8 * flow.shape[2], 8 * flow.shape[3])
    return 8 * F.interpolate(flow, size=new_size, mode=mode, align_corners=True)
