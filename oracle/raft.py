"""Oracle: full RAFT inference forward on PyTorch-CPU fp32. TEST INFRASTRUCTURE ONLY.

Also the ``cpu_baseline`` timed by ``bench.py`` on the GPU box's host cores (the reference never travels
there). Module structure and ``state_dict`` keys equal the reference's (179 keys), so the same hash weights
load into the reference, this oracle and the product model.
"""
from __future__ import annotations

from typing import List, Optional, Sequence, Tuple

import torch
import torch.nn as nn
import torch.nn.functional as F

from oracle.corr import coords_grid, corr_lookup, corr_pyramid


def _norm(kind: str, ch: int) -> nn.Module:
    if kind == "group":
        return nn.GroupNorm(num_groups=ch // 8, num_channels=ch)
    if kind == "batch":
        return nn.BatchNorm2d(ch)
    if kind == "instance":
        return nn.InstanceNorm2d(ch)
    return nn.Sequential()


class ResidualBlock(nn.Module):
    """conv3x3-norm-relu x2 + (1x1 strided conv + norm) shortcut. `extractor.py:35-90`."""

    def __init__(self, cin: int, cout: int, norm_fn: str, stride: int = 1) -> None:
        super().__init__()
        self.conv1 = nn.Conv2d(cin, cout, 3, padding=1, stride=stride)
        self.conv2 = nn.Conv2d(cout, cout, 3, padding=1)
        self.relu = nn.ReLU(inplace=True)
        gnorm = "group" if norm_fn == "group" else norm_fn
        self.norm1 = _norm(gnorm, cout)
        self.norm2 = _norm(gnorm, cout)
        if stride != 1:
            self.norm3 = _norm(gnorm, cout)
            self.downsample = nn.Sequential(nn.Conv2d(cin, cout, 1, stride=stride), self.norm3)
        else:
            self.downsample = None

    def forward(self, x):
        y = self.relu(self.norm1(self.conv1(x)))
        y = self.relu(self.norm2(self.conv2(y)))
        if self.downsample is not None:
            x = self.downsample(x)
        return self.relu(x + y)


class BasicEncoder(nn.Module):
    """7x7/2 stem, 3 stages of 2 residual blocks (64, 96/2, 128/2), 1x1 head. `extractor.py:156-231`."""

    def __init__(self, output_dim: int = 128, norm_fn: str = "batch") -> None:
        super().__init__()
        self.norm_fn = norm_fn
        self.norm1 = nn.GroupNorm(8, 64) if norm_fn == "group" else _norm(norm_fn, 64)
        self.conv1 = nn.Conv2d(3, 64, 7, stride=2, padding=3)
        self.relu1 = nn.ReLU(inplace=True)
        self.in_planes = 64
        self.layer1 = self._layer(64, 1)
        self.layer2 = self._layer(96, 2)
        self.layer3 = self._layer(128, 2)
        self.conv2 = nn.Conv2d(128, output_dim, 1)

    def _layer(self, dim: int, stride: int) -> nn.Module:
        blocks = nn.Sequential(
            ResidualBlock(self.in_planes, dim, self.norm_fn, stride), ResidualBlock(dim, dim, self.norm_fn, 1)
        )
        self.in_planes = dim
        return blocks

    def forward(self, x):
        is_list = isinstance(x, (list, tuple))
        if is_list:
            n = x[0].shape[0]
            x = torch.cat(x, dim=0)
        x = self.relu1(self.norm1(self.conv1(x)))
        x = self.conv2(self.layer3(self.layer2(self.layer1(x))))
        if is_list:
            return torch.split(x, [n, n], dim=0)
        return x


class FlowHead(nn.Module):
    """`update.py:40-48`."""

    def __init__(self, input_dim: int = 128, hidden_dim: int = 256) -> None:
        super().__init__()
        self.conv1 = nn.Conv2d(input_dim, hidden_dim, 3, padding=1)
        self.conv2 = nn.Conv2d(hidden_dim, 2, 3, padding=1)
        self.relu = nn.ReLU(inplace=True)

    def forward(self, x):
        return self.conv2(self.relu(self.conv1(x)))


class SepConvGRU(nn.Module):
    """Horizontal (1x5) then vertical (5x1) GRU. `update.py:69-107`."""

    def __init__(self, hidden_dim: int = 128, input_dim: int = 192 + 128) -> None:
        super().__init__()
        c = hidden_dim + input_dim
        for tag, k, p in (("1", (1, 5), (0, 2)), ("2", (5, 1), (2, 0))):
            for g in "zrq":
                setattr(self, f"conv{g}{tag}", nn.Conv2d(c, hidden_dim, k, padding=p))

    def _half(self, h, x, tag):
        hx = torch.cat([h, x], dim=1)
        z = torch.sigmoid(getattr(self, f"convz{tag}")(hx))
        r = torch.sigmoid(getattr(self, f"convr{tag}")(hx))
        q = torch.tanh(getattr(self, f"convq{tag}")(torch.cat([r * h, x], dim=1)))
        return (1 - z) * h + z * q

    def forward(self, h, x):
        return self._half(self._half(h, x, "1"), x, "2")


class BasicMotionEncoder(nn.Module):
    """`update.py:110-128`."""

    def __init__(self, corr_levels: int, corr_radius: int) -> None:
        super().__init__()
        planes = corr_levels * (2 * corr_radius + 1) ** 2
        self.convc1 = nn.Conv2d(planes, 256, 1)
        self.convc2 = nn.Conv2d(256, 192, 3, padding=1)
        self.convf1 = nn.Conv2d(2, 128, 7, padding=3)
        self.convf2 = nn.Conv2d(128, 64, 3, padding=1)
        self.conv = nn.Conv2d(64 + 192, 128 - 2, 3, padding=1)

    def forward(self, flow, corr):
        cor = F.relu(self.convc2(F.relu(self.convc1(corr))))
        flo = F.relu(self.convf2(F.relu(self.convf1(flow))))
        out = F.relu(self.conv(torch.cat([cor, flo], dim=1)))
        return torch.cat([out, flow], dim=1)


class BasicUpdateBlock(nn.Module):
    """`update.py:131-161` (mask scaled by 0.25)."""

    def __init__(self, corr_levels: int, corr_radius: int, hidden_dim: int = 128) -> None:
        super().__init__()
        self.encoder = BasicMotionEncoder(corr_levels, corr_radius)
        self.gru = SepConvGRU(hidden_dim=hidden_dim, input_dim=128 + hidden_dim)
        self.flow_head = FlowHead(hidden_dim, hidden_dim=256)
        self.mask = nn.Sequential(nn.Conv2d(128, 256, 3, padding=1), nn.ReLU(inplace=True), nn.Conv2d(256, 64 * 9, 1))

    def forward(self, net, inp, corr, flow):
        inp = torch.cat([inp, self.encoder(flow, corr)], dim=1)
        net = self.gru(net, inp)
        return net, 0.25 * self.mask(net), self.flow_head(net)


def upsample_flow(flow: torch.Tensor, mask: torch.Tensor) -> torch.Tensor:
    """Convex 8x upsampling: softmax over 9 neighbours of unfold(8*flow). `raft.py:73-85`."""
    n, _, h, w = flow.shape
    mask = torch.softmax(mask.view(n, 1, 9, 8, 8, h, w), dim=2)
    up = F.unfold(8 * flow, [3, 3], padding=1).view(n, 2, 9, 1, 1, h, w)
    up = torch.sum(mask * up, dim=2).permute(0, 1, 4, 2, 5, 3)
    return up.reshape(n, 2, 8 * h, 8 * w)


class InputPadder:
    """Replicate-pad to a multiple of 8; 'sintel' pads both sides, other modes bottom only. `utils.py:38-61`."""

    def __init__(self, dims: Sequence[int], mode: str = "sintel") -> None:
        self.ht, self.wd = dims[-2:]
        ph = (((self.ht // 8) + 1) * 8 - self.ht) % 8
        pw = (((self.wd // 8) + 1) * 8 - self.wd) % 8
        if mode == "sintel":
            self._pad = [pw // 2, pw - pw // 2, ph // 2, ph - ph // 2]
        else:
            self._pad = [pw // 2, pw - pw // 2, 0, ph]

    def pad(self, *inputs: torch.Tensor) -> List[torch.Tensor]:
        return [F.pad(x, self._pad, mode="replicate") for x in inputs]

    def unpad(self, x: torch.Tensor) -> torch.Tensor:
        ht, wd = x.shape[-2:]
        return x[..., self._pad[2] : ht - self._pad[3], self._pad[0] : wd - self._pad[1]]


class RAFT(nn.Module):
    """RAFT forward. `raft.py:21-147`. ``num_levels`` of the pyramid is always 4 (Q7, `raft.py:112`)."""

    def __init__(self, hidden_dim: int = 128, context_dim: int = 128, corr_levels: int = 4, corr_radius: int = 4):
        super().__init__()
        self.hidden_dim, self.context_dim, self.corr_radius = hidden_dim, context_dim, corr_radius
        self.fnet = BasicEncoder(256, "instance")
        self.cnet = BasicEncoder(hidden_dim + context_dim, "batch")
        self.update_block = BasicUpdateBlock(corr_levels, corr_radius, hidden_dim)

    def forward(self, image0, image1, iters: int = 12, flow_init: Optional[torch.Tensor] = None, test_mode=False):
        image0 = (2 * (image0 / 255.0) - 1.0).contiguous()
        image1 = (2 * (image1 / 255.0) - 1.0).contiguous()
        fmap1, fmap2 = self.fnet([image0, image1])
        pyramid = corr_pyramid(fmap1.float(), fmap2.float(), 4)
        net, inp = torch.split(self.cnet(image0), [self.hidden_dim, self.context_dim], dim=1)
        net, inp = torch.tanh(net), torch.relu(inp)
        n, _, h, w = image0.shape
        coords0 = coords_grid(n, h // 8, w // 8).to(image0.device)
        coords1 = coords_grid(n, h // 8, w // 8).to(image0.device)
        if flow_init is not None:
            coords1 = coords1 + flow_init
        preds = []
        flow_up = None
        for _ in range(iters):
            coords1 = coords1.detach()  # raft.py:127 (no effect on the values; gradients stop here as in the reference)
            corr = corr_lookup(pyramid, coords1, self.corr_radius)
            net, up_mask, delta = self.update_block(net, inp, corr, coords1 - coords0)
            coords1 = coords1 + delta
            flow_up = upsample_flow(coords1 - coords0, up_mask)
            preds.append(flow_up)
        if test_mode:
            return coords1 - coords0, flow_up
        return preds


def end_point_error(pred: torch.Tensor, target: torch.Tensor, dim: int = 1) -> torch.Tensor:
    """Per-pixel L2 norm of the residual. `optical_flow/metrics/epe.py:41-61`."""
    return torch.norm(pred - target, p=2, dim=dim)
