"""Feature / context encoders (reference: methods/raft/model/extractor.py:35-231).

``BasicEncoder``/``ResidualBlock`` are the nn.Modules (parameter names and registration order equal the
reference's, so reference ``state_dict``s load unchanged). For GPU inference RAFT runs them through
``SplitEncoder``: every convolution on the split-fp16 matrix-core kernel (csrc/conv_s32.hip), instance norm from
per-tile partials merged in fp64, batch norm (eval) folded into the convolutions, ReLU / residual adds fused, and the
stride-2 stages fed in space-to-depth layout. ``SmallEncoder``/``BottleneckBlock`` (never instantiated by RAFT,
`raft.py:40-47`) are not provided.
"""
from __future__ import annotations

import os

from typing import Optional, List, Sequence, Tuple, Union

import torch
import torch.nn as nn
from torch import Tensor

from optical_flow import _native

from .update import CONV_BLOCKS, parse_block_overrides


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


# ---- split-fp16 inference path ---------------------------------------------------------------------------------


def _s2d_weight(w: Tensor) -> Tensor:
    """(N, C, 3, 3) stride-2 pad-1 weights -> (N, 4C, 2, 2) stride-1 weights over the space-to-depth input (channel
    (a*2 + b)*C + c = input pixel (2Y + a, 2X + b)); taps at offsets -1, 0: ky = 2*ky' + a - 1."""
    n, c = w.shape[:2]
    out = torch.zeros((n, 4, c, 2, 2), device=w.device, dtype=w.dtype)
    for kyp in range(2):
        for a in range(2):
            ky = 2 * kyp + a - 1
            if not 0 <= ky <= 2:
                continue
            for kxp in range(2):
                for b in range(2):
                    kx = 2 * kxp + b - 1
                    if 0 <= kx <= 2:
                        out[:, a * 2 + b, :, kyp, kxp] = w[:, :, ky, kx]
    return out.reshape(n, 4 * c, 2, 2)


def _fold_bn(conv: nn.Conv2d, bn: nn.Module):
    """Eval-mode BatchNorm after a conv folded into it (ATen: y = x*alpha + beta, alpha = gamma/sqrt(var + eps),
    beta = beta - mean*alpha), computed in fp64."""
    w = conv.weight.detach().double()
    b = conv.bias.detach().double() if conv.bias is not None else torch.zeros(w.shape[0], device=w.device, dtype=w.dtype)
    alpha = bn.weight.detach().double() / torch.sqrt(bn.running_var.detach().double() + bn.eps)
    beta = bn.bias.detach().double() - bn.running_mean.detach().double() * alpha
    return (w * alpha.view(-1, 1, 1, 1)).float(), (b * alpha + beta).float()


# (A/B runs: OFLOW_ENC_BN="128=64,96=32" maps the encoder convs' default output-channel blocks to others)
_ENC_BN_OVERRIDE = {int(k): v for k, v in
                    parse_block_overrides("OFLOW_ENC_BN", {str(b) for b in CONV_BLOCKS}).items()}


class SplitEncoder:
    """Inference execution of a ``BasicEncoder`` (norm 'instance' or 'batch' in eval mode) on the split-fp16 kernels.

    Activations are S32 (split-fp16 NHWC, include/oflow.h). Instance norm: each conv writes its fp32 NHWC output plus
    per-tile (count, mean, M2) partials; ``oflow_norm_stats_finalize`` merges them in fp64 and ``oflow_norm_apply_s32``
    applies x*invstd - mean*invstd, the ReLU and the block's residual tail. Batch norm: folded into the conv, ReLU and
    the residual add run in the conv epilogue. Stride-2 3x3 convs run as 2x2 convs on the space-to-depth layout that
    the previous stage writes directly; their 1x1 stride-2 shortcuts read its first C channels. The stem is a 1x1 GEMM
    over the 7x7 patch matrix.
    """

    def __init__(self, enc: BasicEncoder) -> None:
        if enc.norm_fn not in ("instance", "batch"):
            raise RuntimeError(f"SplitEncoder: norm_fn {enc.norm_fn!r} not supported")
        if enc.norm_fn == "batch" and enc.training:
            raise RuntimeError("SplitEncoder: batch norm needs eval mode (running statistics)")
        self.enc = enc
        self.inorm = enc.norm_fn == "instance"
        from .update import cached_pack, tensor_key

        key = tuple(tensor_key(q) for q in enc.parameters()) + tuple(tensor_key(q) for q in enc.buffers())
        self.w = cached_pack(enc, key, lambda: self._pack(enc))

    def _cw(self, conv: nn.Conv2d, norm, **kw):
        if self.inorm or norm is None:
            w, b = conv.weight, conv.bias
        else:
            w, b = _fold_bn(conv, norm)
        if kw.pop("s2d", False):
            w = _s2d_weight(w.detach().float())
        n = w.shape[0]
        return _native.ConvWeights(w, b, ((n + 31) // 32) * 32, **kw)

    def _pack(self, enc: BasicEncoder):
        W = {"stem": self._cw(enc.conv1, enc.norm1, patches=True)}
        for li, layer in enumerate((enc.layer1, enc.layer2, enc.layer3)):
            for bi, blk in enumerate(layer):
                s2 = blk.downsample is not None
                W[f"{li}.{bi}.conv1"] = self._cw(blk.conv1, blk.norm1, s2d=s2)
                W[f"{li}.{bi}.conv2"] = self._cw(blk.conv2, blk.norm2)
                if s2:
                    W[f"{li}.{bi}.down"] = self._cw(blk.downsample[0], blk.downsample[1])
        W["head"] = _native.ConvWeights(enc.conv2.weight, enc.conv2.bias, ((enc.conv2.out_channels + 31) // 32) * 32)
        return W

    @staticmethod
    def _bn(n: int) -> int:
        bn = {64: 64, 96: 96, 128: 128}.get(n, 128 if n % 128 == 0 else 64 if n % 64 == 0 else 32)
        return _ENC_BN_OVERRIDE.get(bn, bn)

    def _conv_norm(self, x, cw, shape, act, out=None, res=None, s2d=False, raw_only=False):
        """conv -> norm -> act [-> + res -> relu]: returns the S32 output (or (raw, alpha, beta) when raw_only)."""
        b, h, w = shape
        bn = self._bn(cw.n)
        V = _native.S32Slice
        dev = x.device
        if self.inorm:
            raw = torch.empty((b * h * w, cw.n), device=dev, dtype=torch.float32)
            tiles = _native.conv_tiles(h, w)
            part = torch.empty((b, tiles, cw.n_pad, 3), device=dev, dtype=torch.float32)
            _native.conv_s32(x, cw, bn, nhwc=raw, stats=part)
            alpha, beta = _native.norm_stats(part, b, tiles, cw.n_pad, cw.n, 1e-5)
            if raw_only:
                return raw, alpha, beta
            if out is None:
                out = _native.s32_empty(b, h // 2 if s2d else h, w // 2 if s2d else w, (cw.n * (4 if s2d else 1) + 31) // 32, dev)
            if isinstance(res, _native.NhwcNormIn):  # a block input kept raw: relu(norm(x)) + y
                _native.norm_apply(raw, (b, cw.n, h, w), alpha, beta, act, V(out), res_raw=(res.raw, res.scale, res.shift),
                                   res_act="relu", s2d=s2d, res_raw_relu=True)
            elif isinstance(res, tuple):
                _native.norm_apply(raw, (b, cw.n, h, w), alpha, beta, act, V(out), res_raw=res, res_act="relu", s2d=s2d)
            else:
                _native.norm_apply(raw, (b, cw.n, h, w), alpha, beta, act, V(out), res=res, res_act="relu" if res is not None else "none", s2d=s2d)
            return out
        if raw_only:
            out = _native.s32_empty(b, h, w, (cw.n + 31) // 32, dev)
            _native.conv_s32(x, cw, bn, y0=V(out))
            return out
        if out is None:
            out = _native.s32_empty(b, h // 2 if s2d else h, w // 2 if s2d else w, (cw.n * (4 if s2d else 1) + 31) // 32, dev)
        _native.conv_s32(x, cw, bn, act=act, y0=V(out), res=res, res_act="relu" if res is not None else "none", s2d=s2d)
        return out

    def _conv1(self, x, cw, shape):
        """A residual block's first conv -> relu(norm1(.)) as the second conv's input: with instance norm the raw
        fp32 output and its statistics (normalised + ReLU'd while the next conv stages it, oflow_conv_s32_ex2); with
        folded batch norm an S32 tensor."""
        if self.inorm:
            raw, alpha, beta = self._conv_norm(x, cw, shape, "relu", raw_only=True)
            return _native.NhwcNormIn(raw, *shape, alpha, beta)
        return _native.S32Slice(self._conv_norm(x, cw, shape, "relu"))

    def stem_patches(self, x: Tensor) -> Tensor:
        """The stem's 7x7/2 patch matrix (S32) of a (n, 3, H, W) input, as ``__call__`` would build it."""
        x = x.float().contiguous()
        n, _, hh, ww = x.shape
        patches = _native.s32_empty(n, hh // 2, ww // 2, self.w["stem"].kg, x.device)
        _native.stem_patches(x, patches)
        return patches

    def __call__(self, x: Union[Tensor, Sequence[Tensor]], patches: Optional[Tensor] = None,
                 split_out: bool = False, stem_from_image: bool = False) -> Union[Tensor, Tuple[Tensor, ...]]:
        """``patches``: the stem's patch matrix of ``x`` when another encoder already built it (RAFT's cnet reads
        image0's rows of fnet's, raft.py:109/115); the one built here is kept as ``self.patches``. ``split_out``: the
        head convolution writes its output as S32 rows (B, H, W, C/32, 2, 32) instead of fp32 NCHW (the RAFT forward's
        correlation input, CorrBlock.from_split_features). ``stem_from_image``: the stem convolution builds its 7x7
        patch operand from the image tile by tile (OFLOW_IN_IMG7S2) instead of reading a patch matrix (none is
        written; ``patches`` is ignored)."""
        is_list = isinstance(x, (tuple, list))
        if is_list:
            batch_dim = x[0].shape[0]
            n, _, hh, ww = x[0].shape
            n *= len(x)
            if patches is None or tuple(patches.shape[:4]) != (n, hh // 2, ww // 2, self.w["stem"].kg):
                x = torch.cat(list(x), dim=0)  # (with the patches given the images themselves are not read)
        if not isinstance(x, (tuple, list)):
            x = x.float().contiguous()
            n, _, hh, ww = x.shape
            dev = x.device
        else:
            dev = x[0].device
        if hh % 8 or ww % 8:
            raise RuntimeError("SplitEncoder: H and W must be multiples of 8")
        V = _native.S32Slice
        h, w = hh // 2, ww // 2
        if stem_from_image:
            if isinstance(x, (tuple, list)):
                x = torch.cat([t.float() for t in x], dim=0)
            stem_in = _native.ImgIn(x.float().contiguous())
            self.patches = None
        else:
            if patches is None or tuple(patches.shape[:4]) != (n, h, w, self.w["stem"].kg):
                patches = _native.s32_empty(n, h, w, self.w["stem"].kg, dev)
                _native.stem_patches(x, patches)
            self.patches = patches
            stem_in = V(patches)
        # instance norm: the stem's output stays raw fp32 + its norm (relu(norm(.)) applied by layer1's first conv while
        # it stages its input, and by that block's residual tail): no normalised copy is written
        cur = (self._conv1(stem_in, self.w["stem"], (n, h, w)) if self.inorm
               else self._conv_norm(stem_in, self.w["stem"], (n, h, w), "relu"))
        layers = (self.enc.layer1, self.enc.layer2, self.enc.layer3)
        for li, layer in enumerate(layers):
            for bi, blk in enumerate(layer):
                last_of_stage = bi == len(layer) - 1
                out_s2d = last_of_stage and li + 1 < len(layers)  # the next stage starts with stride-2 convs
                pre = f"{li}.{bi}."
                if blk.downsample is None:
                    x_in = cur if isinstance(cur, _native.NhwcNormIn) else V(cur)
                    t = self._conv1(x_in, self.w[pre + "conv1"], (n, h, w))
                    cur = self._conv_norm(t, self.w[pre + "conv2"], (n, h, w), "relu", res=x_in, s2d=out_s2d)
                else:
                    h, w = h // 2, w // 2  # cur is the space-to-depth input at the new resolution
                    t = self._conv1(V(cur), self.w[pre + "conv1"], (n, h, w))
                    cin = self.w[pre + "down"].kg
                    d = self._conv_norm(V(cur, 0, cin), self.w[pre + "down"], (n, h, w), "none", raw_only=True)
                    res = d if self.inorm else V(d)
                    cur = self._conv_norm(t, self.w[pre + "conv2"], (n, h, w), "relu", res=res, s2d=out_s2d)
                if out_s2d:
                    pass  # cur now holds (n, h/2, w/2, 4C) for the next stage
        head = self.w["head"]
        if split_out:
            out = _native.s32_empty(n, h, w, (head.n + 31) // 32, dev)
            _native.conv_s32(V(cur), head, self._bn(head.n), y0=V(out))
        else:
            out = torch.empty((n, head.n, h, w), device=dev, dtype=torch.float32)
            _native.conv_s32(V(cur), head, self._bn(head.n), f32=out)
        if is_list:
            return torch.split(out, [batch_dim, batch_dim], dim=0)
        return out
