"""Feature / context encoders (reference: methods/raft/model/extractor.py:35-231).

Caller-side of the hot path: the convolutions run on PyTorch-ROCm (MIOpen), not on custom kernels in this
build. Parameter names and registration order equal the reference's, so reference
``state_dict``s load unchanged. ``SmallEncoder``/``BottleneckBlock`` (never instantiated by RAFT,
`raft.py:40-47`) are not provided.
"""
from __future__ import annotations

from typing import List, Sequence, Tuple, Union

import torch
import torch.nn as nn
from torch import Tensor


def _norm_layer(norm_fn: str, planes: int, groups: int) -> nn.Module:
    if norm_fn == "group":
        return nn.GroupNorm(num_groups=groups, num_channels=planes)
    if norm_fn == "batch":
        return nn.BatchNorm2d(planes)
    if norm_fn == "instance":
        return nn.InstanceNorm2d(planes)
    if norm_fn == "none":
        return nn.Sequential()
    raise ValueError(f"unknown norm_fn {norm_fn!r}")


class ResidualBlock(nn.Module):
    """Two 3x3 conv + norm + ReLU with an optional strided 1x1 projection (`extractor.py:35-90`)."""

    def __init__(self, in_planes: int, planes: int, norm_fn: str = "group", stride: int = 1) -> None:
        super().__init__()
        self.conv1 = nn.Conv2d(in_planes, planes, kernel_size=3, padding=1, stride=stride)
        self.conv2 = nn.Conv2d(planes, planes, kernel_size=3, padding=1)
        self.relu = nn.ReLU(inplace=True)
        groups = planes // 8
        self.norm1 = _norm_layer(norm_fn, planes, groups)
        self.norm2 = _norm_layer(norm_fn, planes, groups)
        if stride != 1:
            self.norm3 = _norm_layer(norm_fn, planes, groups)
            self.downsample = nn.Sequential(nn.Conv2d(in_planes, planes, kernel_size=1, stride=stride), self.norm3)
        else:
            self.downsample = None

    def forward(self, x: Tensor) -> Tensor:
        y = self.relu(self.norm1(self.conv1(x)))
        y = self.relu(self.norm2(self.conv2(y)))
        if self.downsample is not None:
            x = self.downsample(x)
        return self.relu(x + y)


class BasicEncoder(nn.Module):
    """7x7/2 stem (64) -> residual stages 64, 96 (/2), 128 (/2) -> 1x1 to ``output_dim`` at 1/8 resolution
    (`extractor.py:156-231`). A list/tuple input is concatenated on the batch axis and split back after."""

    def __init__(self, output_dim: int = 128, norm_fn: str = "batch", dropout: float = 0.0) -> None:
        super().__init__()
        self.norm_fn = norm_fn
        self.norm1 = _norm_layer(norm_fn, 64, 8)
        self.conv1 = nn.Conv2d(3, 64, kernel_size=7, stride=2, padding=3)
        self.relu1 = nn.ReLU(inplace=True)
        self.in_planes = 64
        self.layer1 = self._make_layer(64, stride=1)
        self.layer2 = self._make_layer(96, stride=2)
        self.layer3 = self._make_layer(128, stride=2)
        self.conv2 = nn.Conv2d(128, output_dim, kernel_size=1)
        self.dropout = nn.Dropout2d(p=dropout) if dropout > 0 else None
        for m in self.modules():
            if isinstance(m, nn.Conv2d):
                nn.init.kaiming_normal_(m.weight, mode="fan_out", nonlinearity="relu")
            elif isinstance(m, (nn.BatchNorm2d, nn.InstanceNorm2d, nn.GroupNorm)):
                if m.weight is not None:
                    nn.init.constant_(m.weight, 1)
                if m.bias is not None:
                    nn.init.constant_(m.bias, 0)

    def _make_layer(self, dim: int, stride: int = 1) -> nn.Module:
        blocks = (ResidualBlock(self.in_planes, dim, self.norm_fn, stride=stride), ResidualBlock(dim, dim, self.norm_fn, 1))
        self.in_planes = dim
        return nn.Sequential(*blocks)

    def forward(self, x: Union[Tensor, Sequence[Tensor]]) -> Union[Tensor, Tuple[Tensor, ...]]:
        is_list = isinstance(x, (tuple, list))
        if is_list:
            batch_dim = x[0].shape[0]
            x = torch.cat(list(x), dim=0)
        x = self.relu1(self.norm1(self.conv1(x)))
        x = self.layer3(self.layer2(self.layer1(x)))
        x = self.conv2(x)
        if self.training and self.dropout is not None:
            x = self.dropout(x)
        if is_list:
            return torch.split(x, [batch_dim, batch_dim], dim=0)
        return x
