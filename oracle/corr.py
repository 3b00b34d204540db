"""Oracle: all-pairs correlation pyramid and its windowed bilinear lookup on PyTorch-CPU fp32.

TEST INFRASTRUCTURE ONLY (see ``oracle/__init__.py``).
"""
from __future__ import annotations

from typing import List, Sequence

import numpy as np
import torch
import torch.nn.functional as F


def coords_grid(batch: int, ht: int, wd: int) -> torch.Tensor:
    """(B, 2, ht, wd) with channel 0 = x (column), channel 1 = y (row). `utils.py:83-86`."""
    ys, xs = torch.meshgrid(torch.arange(ht), torch.arange(wd), indexing="ij")
    return torch.stack((xs, ys), dim=0).float()[None].repeat(batch, 1, 1, 1)


def corr_volume(fmap1: torch.Tensor, fmap2: torch.Tensor) -> torch.Tensor:
    """corr[b, i, j] = <f1[:, i], f2[:, j]> / sqrt(C), shaped (B, H, W, 1, H, W). `corr.py:79-87`."""
    b, c, h, w = fmap1.shape
    a = fmap1.reshape(b, c, h * w).transpose(1, 2)
    m = torch.matmul(a, fmap2.reshape(b, c, h * w))
    return m.view(b, h, w, 1, h, w) / torch.sqrt(torch.tensor(c).float())


def corr_pyramid(fmap1: torch.Tensor, fmap2: torch.Tensor, num_levels: int = 4) -> List[torch.Tensor]:
    """Level 0 reshaped to (B*H*W, 1, H, W), then ``num_levels-1`` floor 2x2 average pools. `corr.py:38-54`."""
    corr = corr_volume(fmap1, fmap2)
    b, h1, w1, d, h2, w2 = corr.shape
    lvl = corr.reshape(b * h1 * w1, d, h2, w2)
    pyr = [lvl]
    for _ in range(num_levels - 1):
        lvl = F.avg_pool2d(lvl, 2, stride=2)
        pyr.append(lvl)
    return pyr


def bilinear_sampler(img: torch.Tensor, coords: torch.Tensor) -> torch.Tensor:
    """grid_sample with pixel coordinates, align_corners=True, zeros padding. `utils.py:64-80`."""
    h, w = img.shape[-2:]
    x, y = coords[..., :1], coords[..., 1:]
    grid = torch.cat([2 * x / (w - 1) - 1, 2 * y / (h - 1) - 1], dim=-1)
    return F.grid_sample(img, grid, align_corners=True)


def corr_lookup(pyramid: Sequence[torch.Tensor], coords: torch.Tensor, radius: int = 4) -> torch.Tensor:
    """(B, L*(2r+1)^2, H, W) fp32 windowed lookup. `corr.py:56-77`.

    Window channel k = l*(2r+1)^2 + i*(2r+1) + j samples at (x + i - r, y + j - r): the delta grid is
    ``stack(meshgrid(dy, dx))`` added to (x, y), so the FIRST window index moves x.
    """
    r = radius
    b, _, h1, w1 = coords.shape
    cent = coords.permute(0, 2, 3, 1).reshape(b * h1 * w1, 1, 1, 2)
    d = torch.linspace(-r, r, 2 * r + 1)
    dy, dx = torch.meshgrid(d, d, indexing="ij")
    delta = torch.stack((dy, dx), dim=-1).view(1, 2 * r + 1, 2 * r + 1, 2).to(coords.device)
    outs = []
    for i, lvl in enumerate(pyramid):
        sampled = bilinear_sampler(lvl, cent / 2**i + delta)
        outs.append(sampled.view(b, h1, w1, -1))
    return torch.cat(outs, dim=-1).permute(0, 3, 1, 2).contiguous().float()


def corr_lookup_f64(pyramid: Sequence[np.ndarray], coords: np.ndarray, radius: int = 4) -> np.ndarray:
    """Independent float64 restatement in pixel space; small inputs only.

    For query q and level l: c = coords/2^l, x0 = floor(cx), wx = cx - x0 (shared by all window taps), then
    out[l*(2r+1)^2 + i*(2r+1) + j] = bilinear(P, x0 + i - r + wx, y0 + j - r + wy), zero outside the level.
    """
    r = radius
    k = 2 * r + 1
    b, _, h1, w1 = coords.shape
    n = h1 * w1
    out = np.zeros((b, len(pyramid) * k * k, h1, w1), dtype=np.float64)
    cx_all = coords[:, 0].reshape(b, n).astype(np.float64)
    cy_all = coords[:, 1].reshape(b, n).astype(np.float64)
    for lvl, p in enumerate(pyramid):
        p = np.asarray(p, dtype=np.float64).reshape(b, n, p.shape[-2], p.shape[-1])
        hl, wl = p.shape[-2:]
        pad = np.zeros((b, n, hl + 2 * k + 2, wl + 2 * k + 2))
        pad[:, :, k + 1 : k + 1 + hl, k + 1 : k + 1 + wl] = p
        cx, cy = cx_all / 2**lvl, cy_all / 2**lvl
        x0, y0 = np.floor(cx), np.floor(cy)
        wx, wy = cx - x0, cy - y0
        for bi in range(b):
            for q in range(n):
                xs, ys = int(x0[bi, q]) - r, int(y0[bi, q]) - r
                if not (-(k + 1) <= xs <= wl and -(k + 1) <= ys <= hl):
                    continue  # window entirely outside: all taps are zero padding
                patch = pad[bi, q, ys + k + 1 : ys + 2 * k + 2, xs + k + 1 : xs + 2 * k + 2]  # (k+1, k+1)
                ax, ay = wx[bi, q], wy[bi, q]
                hor = (1 - ax) * patch[:, :-1] + ax * patch[:, 1:]  # (k+1, k) over j-rows, i-cols
                s = (1 - ay) * hor[:-1, :] + ay * hor[1:, :]  # s[j, i]
                out[bi, lvl * k * k : (lvl + 1) * k * k, q // w1, q % w1] = s.T.reshape(-1)
    return out
