"""GRU update block (reference: methods/raft/model/update.py:40-161).

The ``nn.Module`` classes restate the reference's layers (same parameter names, so checkpoints load); they are
what autograd / CPU runs use. GPU inference runs ``SplitUpdate``: every convolution on the split-fp16 matrix-core
kernel (csrc/conv_s32.hip) with the GRU gates, activations, concatenations and the coords update fused into
convolution epilogues; the correlation lookup runs inside convc1 (csrc/corr_convc1.hip).
``FusedUpdate`` (MIOpen convolutions + fused elementwise kernels) is kept for A/B runs. ``ConvGRU`` (unused by RAFT)
is not provided.
"""
from __future__ import annotations

import contextlib
import os
import threading
from typing import Optional, Tuple

import torch
import torch.nn as nn
import torch.nn.functional as F
from torch import Tensor

from optical_flow import _native



# output-channel block (workgroup N) per update-block conv of the split path; tools/exp/run_conv_bn_ab.py A/Bs them
# output-channel block per update-block conv. r05 re-check on the graph bench (profiles/r05/s43-s45, alternated on one
# box each): convc2 96 (two 96-channel blocks, each wave 32 px x 96 ch: 8 operand reads per 9 MFMA triples instead of
# 6 per 6, the halo staged twice instead of three times) +2.0 %; with the flow head's first conv at 64 (LDS-staged
# 64-channel blocks, 880 workgroups per lane) 444.2 / 444.8 / 444.8 vs 444.3 / 441.1 / 442.7 pairs/s for convc2 96
# alone; the motion conv at 64 is +1.5 % alone but not on top of convc2 96, convf2 at 32 -2 %. Bit-identical (the
# K order per output is the same for every block). Those runs replay the graph, whose lanes run the flow branch inline
# (model/graph.py); with the flow branch on a side stream beside convc1 -> convc2 (the eager forward) the same blocks
# cost 1.2 % (eager 428.8 / 427.7 / 427.4 vs 432.2 / 434.7 / 432.4 pairs/s, s51), so that case keeps the r04 blocks
# (CONV_BN_SIDE).
CONV_BN = {"c2": 96, "f1": 128, "f2": 64, "mo": 128, "gru": 128, "fh1": 64}
CONV_BN_SIDE = dict(CONV_BN, c2=64, fh1=128)
CONV_BLOCKS = (32, 64, 96, 128)  # output-channel blocks conv_s32 instantiates


def parse_block_overrides(var: str, keys) -> dict:
    """An A/B override "k1=v1,k2=v2" from environment variable ``var``, validated at import: every key one of ``keys``,
    every value a conv block of ``CONV_BLOCKS``; anything else raises ValueError naming the variable."""
    spec = os.environ.get(var, "")
    out = {}
    for kv in filter(None, (s.strip() for s in spec.split(","))):
        k, sep, v = kv.partition("=")
        if not sep or not v.strip().isdigit():
            raise ValueError(f"{var}={spec!r}: expected comma-separated key=block entries, got {kv!r}")
        key = k.strip()
        if keys is not None and key not in keys:
            raise ValueError(f"{var}={spec!r}: unknown key {key!r} (one of {sorted(keys)})")
        if int(v) not in CONV_BLOCKS:
            raise ValueError(f"{var}={spec!r}: block {v} for {key!r} is not one of {CONV_BLOCKS}")
        out[key] = int(v)
    return out


def _env_choice(var: str, default: str, choices) -> str:
    v = os.environ.get(var, default)
    if v not in choices:
        raise ValueError(f"{var}={v!r}: expected one of {list(choices)}")
    return v


# (A/B runs only: OFLOW_CONV_BN="c2=96,mo=64" overrides entries of both)
for _bn in (CONV_BN, CONV_BN_SIDE):
    _bn.update(parse_block_overrides("OFLOW_CONV_BN", set(CONV_BN)))
# the flow head's output conv (3x3, 256 -> 2) above the small-grid threshold: "conv" = the 3x3 conv with 2 of its 32
# output columns used, coords1 += in its epilogue; "col2im" = a 1x1 conv 256 -> 18 (the 9 taps' products at the input
# pixel, 18 of 32 MFMA columns used) + a gather of the 9 taps into coords1 (oflow_flow_head_col2im_f32). In-process A/B
# of the 8-pair step: col2im 19.99 / 19.85 ms (median / min) vs conv 19.93 / 19.74 (profiles/r04/s2_ab_fh.log): in the
# step the other pair lane fills the CUs the 2-column conv leaves idle, so "conv" stays the default
# r05: "tiled" = oflow_flow_head2_tiled_s32 (fp32 FMAs on an LDS-staged halo, 512 threads per 4 x 32 tile): step A/B
# 18.81 vs 18.89 ms against "conv" (profiles/r05/s33_flow_head_tiled_ab.log; the first 256-thread form was 0.25 ms
# slower, s32): the default; two channel groups per staging pass: +0.6 % on the graph bench (s37), bit-identical
FLOW_HEAD_MODE = _env_choice("OFLOW_FLOW_HEAD_MODE", "tiled", ("tiled", "conv", "col2im"))
# convf1 (7x7, 2 -> 128) straight from coords1 (_native.FlowIn, OFLOW_IN_FLOW7: each tile stages its flow window and
# builds the patch operand in LDS) from this many pixels of the whole forward's batch up; below it flow_prep writes the
# patch matrix and convf1 runs on the small-grid tiles. Bit-identical either way (same patch values, same k order).
CONVF1_FROM_FLOW_MIN_PIXELS = 16384 if _env_choice("OFLOW_CONVF1_FROM_FLOW", "1", ("0", "1")) == "1" else 1 << 62  # (0: A/B)
# r06: split-K (oflow_conv_s32_ex5) for the update convs whose lane launch fills fewer than half of the chip's
# two-per-CU workgroup slots: the motion conv ("mo", 3x3 256 -> 126) and both GRU candidate convs ("q", 1x5 / 5x1
# 256 -> 128) run 224 workgroups per 4-pair lane unsplit. Each tile's two workgroups sum half of the input groups and
# meet through an fp32 slab (csrc/conv_s32.hip). Decided from the whole forward's pixel count (as the flow head's
# kernel), so pair lanes keep giving the single-lane flows bit for bit. Measured on the replayed 8-pair graph
# (tools/exp/run_graph_ab.py, profiles/r06/r6s12_ab.log, one box, alternated): unsplit 17.73 ms/step, both layers split
# 18.21, q only 17.75, motion only 18.17 -- the other lane's kernels already fill the CUs the 224-workgroup launches
# leave idle, and the split adds a slab round trip and a second workgroup per tile. So the default is unsplit; the
# ex5 path stays for callers whose launches run alone (tests/test_gpu_conv_ksplit.py). e.g. {"mo", "q"} to enable.
KSPLIT_LAYERS = frozenset()
KSPLIT_MIN_PIXELS = 16384

class FlowHead(nn.Module):
    def __init__(self, input_dim: int = 128, hidden_dim: int = 256) -> None:
        super().__init__()
        self.conv1 = nn.Conv2d(input_dim, hidden_dim, 3, padding=1)
        self.conv2 = nn.Conv2d(hidden_dim, 2, 3, padding=1)
        self.relu = nn.ReLU(inplace=True)

    def forward(self, x: Tensor) -> Tensor:
        return self.conv2(self.relu(self.conv1(x)))


class SepConvGRU(nn.Module):
    """GRU with a horizontal (1x5) then a vertical (5x1) pass (`update.py:69-107`)."""

    def __init__(self, hidden_dim: int = 128, input_dim: int = 192 + 128) -> None:
        super().__init__()
        cin = hidden_dim + input_dim
        self.convz1 = nn.Conv2d(cin, hidden_dim, (1, 5), padding=(0, 2))
        self.convr1 = nn.Conv2d(cin, hidden_dim, (1, 5), padding=(0, 2))
        self.convq1 = nn.Conv2d(cin, hidden_dim, (1, 5), padding=(0, 2))
        self.convz2 = nn.Conv2d(cin, hidden_dim, (5, 1), padding=(2, 0))
        self.convr2 = nn.Conv2d(cin, hidden_dim, (5, 1), padding=(2, 0))
        self.convq2 = nn.Conv2d(cin, hidden_dim, (5, 1), padding=(2, 0))

    @staticmethod
    def _step(h: Tensor, x: Tensor, convz: nn.Module, convr: nn.Module, convq: nn.Module) -> Tensor:
        hx = torch.cat([h, x], dim=1)
        z = torch.sigmoid(convz(hx))
        r = torch.sigmoid(convr(hx))
        q = torch.tanh(convq(torch.cat([r * h, x], dim=1)))
        return (1 - z) * h + z * q

    def forward(self, h: Tensor, x: Tensor) -> Tensor:
        h = self._step(h, x, self.convz1, self.convr1, self.convq1)
        return self._step(h, x, self.convz2, self.convr2, self.convq2)


class BasicMotionEncoder(nn.Module):
    """Correlation (1x1 then 3x3) and flow (7x7 then 3x3) branches fused by a 3x3 conv (`update.py:110-128`)."""

    def __init__(self, corr_levels: int, corr_radius: int) -> None:
        super().__init__()
        corr_planes = corr_levels * (2 * corr_radius + 1) ** 2
        self.convc1 = nn.Conv2d(corr_planes, 256, 1, padding=0)
        self.convc2 = nn.Conv2d(256, 192, 3, padding=1)
        self.convf1 = nn.Conv2d(2, 128, 7, padding=3)
        self.convf2 = nn.Conv2d(128, 64, 3, padding=1)
        self.conv = nn.Conv2d(64 + 192, 128 - 2, 3, padding=1)

    def forward(self, flow: Tensor, corr: Tensor) -> Tensor:
        cor = F.relu(self.convc2(F.relu(self.convc1(corr))))
        flo = F.relu(self.convf2(F.relu(self.convf1(flow))))
        out = F.relu(self.conv(torch.cat([cor, flo], dim=1)))
        return torch.cat([out, flow], dim=1)


class BasicUpdateBlock(nn.Module):
    """Motion encoder -> SepConvGRU -> flow head, plus the convex-upsampling mask head x0.25 (`update.py:131-161`)."""

    def __init__(self, corr_levels: int, corr_radius: int, hidden_dim: int = 128) -> None:
        super().__init__()
        self.corr_levels, self.corr_radius = corr_levels, corr_radius
        self.encoder = BasicMotionEncoder(corr_levels, corr_radius)
        self.gru = SepConvGRU(hidden_dim=hidden_dim, input_dim=128 + hidden_dim)
        self.flow_head = FlowHead(hidden_dim, hidden_dim=256)
        self.mask = nn.Sequential(
            nn.Conv2d(128, 256, 3, padding=1), nn.ReLU(inplace=True), nn.Conv2d(256, 64 * 9, 1, padding=0)
        )

    def forward(self, net: Tensor, inp: Tensor, corr: Tensor, flow: Tensor) -> Tuple[Tensor, Tensor, Tensor]:
        motion = self.encoder(flow, corr)
        net = self.gru(net, torch.cat([inp, motion], dim=1))
        delta_flow = self.flow_head(net)
        return net, 0.25 * self.mask(net), delta_flow


class FusedUpdate:
    """Inference-time execution of ``BasicUpdateBlock`` (same weights, same math) with fused elementwise work.

    The GRU state and its input live in two persistent channel-concatenated buffers, ``hx = [h | inp | motion]``
    and ``rhx = [r*h | inp | motion]``, so the four ``torch.cat`` copies per iteration (update.py:93, 96, 100,
    103) and the ``[inp, motion]`` / ``[out, flow]`` cats (update.py:127, 155) disappear: the motion encoder's
    last ReLU writes into both buffers and ``inp`` is written once per forward. Convolutions run on MIOpen without
    bias; bias + activation run as one HIP pass (``oflow_bias_act_f32``). The z and r convolutions of each GRU half
    are one convolution over concatenated weights (the gates are independent output channels), followed by
    ``oflow_gru_reset_f32`` (r*h into ``rhx``) and, after the q convolution, ``oflow_gru_blend_f32`` (h updated
    in place in ``hx``). Requires ROCm tensors and no autograd (it updates its state in place).
    """

    def __init__(self, block: BasicUpdateBlock, net: Tensor, inp: Tensor) -> None:
        b, ch, h, w = net.shape
        self.block, self.ch, self.ci = block, ch, inp.shape[1]
        enc, gru = block.encoder, block.gru
        cm = enc.conv.out_channels + 2
        total = ch + self.ci + cm
        if gru.convz1.in_channels != total:
            raise RuntimeError("FusedUpdate: unexpected GRU input width")
        self.hx = torch.empty((b, total, h, w), device=net.device, dtype=torch.float32)
        self.rhx = torch.empty_like(self.hx)
        self.hx[:, :ch].copy_(net)
        self.hx[:, ch : ch + self.ci].copy_(inp)
        self.rhx[:, ch : ch + self.ci].copy_(inp)
        self.m0 = ch + self.ci  # first motion channel
        self.halves = []
        for tag, pad in (("1", (0, 2)), ("2", (2, 0))):
            cz, cr, cq = (getattr(gru, f"conv{g}{tag}") for g in "zrq")
            wzr = torch.cat([cz.weight, cr.weight], dim=0).contiguous()
            self.halves.append((wzr, cz.bias.contiguous(), cr.bias.contiguous(), cq.weight, cq.bias.contiguous(), pad))

    @staticmethod
    def _conv(x: Tensor, conv: nn.Conv2d) -> Tensor:
        return F.conv2d(x, conv.weight, None, conv.stride, conv.padding, conv.dilation, conv.groups)

    def step(self, corr: Tensor, flow: Tensor, need_mask: bool = True) -> Tuple[Tensor, Optional[Tensor], Tensor]:
        """One update: returns (net, 0.25 * mask(net) or None when ``need_mask`` is False, delta_flow). The mask
        head only feeds the convex upsampling, which test mode needs at the last iteration alone."""
        enc, blk = self.block.encoder, self.block
        cor = _native.bias_act_(self._conv(corr, enc.convc1), enc.convc1.bias, "relu")
        cor = _native.bias_act_(self._conv(cor, enc.convc2), enc.convc2.bias, "relu")
        flo = _native.bias_act_(self._conv(flow, enc.convf1), enc.convf1.bias, "relu")
        flo = _native.bias_act_(self._conv(flo, enc.convf2), enc.convf2.bias, "relu")
        out = self._conv(torch.cat([cor, flo], dim=1), enc.conv)
        m0, m1 = self.m0, self.m0 + out.shape[1]
        _native.bias_act_(out, enc.conv.bias, "relu", out=self.hx[:, m0:m1], out2=self.rhx[:, m0:m1])
        self.hx[:, m1:].copy_(flow)
        self.rhx[:, m1:].copy_(flow)
        h = self.hx[:, : self.ch]
        for wzr, bz, br, wq, bq, pad in self.halves:
            zr = F.conv2d(self.hx, wzr, None, 1, pad)
            _native.gru_reset(zr, br, h, self.rhx[:, : self.ch])
            q = F.conv2d(self.rhx, wq, None, 1, pad)
            _native.gru_blend_(zr, bz, q, bq, h)
        net = h.contiguous()
        fh = blk.flow_head
        delta_flow = fh.conv2(_native.bias_act_(self._conv(net, fh.conv1), fh.conv1.bias, "relu"))
        mask = None
        if need_mask:
            m = _native.bias_act_(self._conv(net, blk.mask[0]), blk.mask[0].bias, "relu")
            mask = _native.bias_act_(self._conv(m, blk.mask[2]), blk.mask[2].bias, "none", scale=0.25)
        return net, mask, delta_flow


class FusedLookup:
    """convc1's input when the lookup runs inside it: the tiled pyramid, the coordinates and the radius."""

    __slots__ = ("pyr", "coords", "radius")

    def __init__(self, pyr, coords: Tensor, radius: int) -> None:
        self.pyr, self.coords, self.radius = pyr, coords, radius


_SIDE_STREAMS = {}


def _side_stream(device: torch.device, slot: int = 0) -> "torch.cuda.Stream":
    """A persistent extra stream per (device, owner stream, slot), reused across forwards. The owner is the stream
    current at the call: forwards issued from different streams (pipelined steps) get disjoint side streams."""
    dev = torch.device(device)
    owner = torch.cuda.current_stream(dev).stream_id
    key = (dev.index, owner, slot)
    if key not in _SIDE_STREAMS:
        _SIDE_STREAMS[key] = torch.cuda.Stream(device=device)
    return _SIDE_STREAMS[key]


_CAPTURE = threading.local()  # per thread: {device index: depth} while GraphedRAFT captures a forward (model/graph.py)


@contextlib.contextmanager
def capturing(device: torch.device):
    """Marks a GraphedRAFT capture of a forward on ``device`` in progress on this thread (see ``capture_active``)."""
    depth = _CAPTURE.__dict__.setdefault("depth", {})
    idx = torch.device(device).index
    depth[idx] = depth.get(idx, 0) + 1
    try:
        yield
    finally:
        depth[idx] -= 1


def capture_active(device: Optional[torch.device] = None) -> bool:
    """Whether a HIP graph capture of a forward on ``device`` (default: the current device) is in progress on this
    thread. Not ``torch.cuda.is_current_stream_capturing()`` alone: a pair lane's stream joins the capture through an
    event wait, and on ROCm such a stream does not report itself as capturing, so a check on it alone let the lane wait
    on an event recorded before the capture -- a dependency the captured graph cannot hold (the two-lane capture crashed
    in capture_end: profiles/r04/s12_graph8.log). Keyed by thread and device: a forward on another thread or device
    while one is captured keeps its weight-cache waits and its range guard."""
    idx = torch.device(device).index if device is not None else torch.cuda.current_device()
    if _CAPTURE.__dict__.get("depth", {}).get(idx, 0) > 0:
        return True
    return torch.cuda.is_current_stream_capturing()


def _module_device(module: nn.Module) -> Optional[torch.device]:
    for p in module.parameters():
        return p.device
    return None


def cached_pack(module: nn.Module, key, build):
    """The packed weights cached on ``module`` for ``key`` (built by ``build()`` on a miss). The packing kernels run on
    the current stream of the module's device at the miss; an event recorded there after them is waited on by every
    later user's current stream of that device, so a forward issued from another stream (pipelined steps) never reads
    weights still being written -- also when the module's GPU is not the current device."""
    dev = _module_device(module)
    on_gpu = dev is not None and dev.type == "cuda"
    cache = module.__dict__.get("_split_weights")
    if cache is not None and cache[0] == key:
        # (not while a graph is being captured: the capture must not depend on an event recorded outside it; a
        # capture follows warm-up forwards and a device sync, so the weights are complete)
        if cache[2] is not None and on_gpu and not capture_active(dev):
            torch.cuda.current_stream(dev).wait_event(cache[2])
        return cache[1]
    if on_gpu:
        with torch.cuda.device(dev):
            w = build()
            ev = torch.cuda.Event()
            ev.record(torch.cuda.current_stream(dev))
    else:
        w, ev = build(), None
    module.__dict__["_split_weights"] = (key, w, ev)
    return w


def tensor_key(q: Tensor):
    """(storage, version) of a weight for the packed-weight caches. Tensors created under torch.inference_mode()
    (e.g. a model built inside an inference-mode function, as predict.py:39 does) have no version counter: they are
    keyed by storage alone."""
    return (q.data_ptr(), -1 if q.is_inference() else q._version)


def _weights_key(block: nn.Module):
    return tuple(tensor_key(q) for q in block.parameters())


class SplitUpdate:
    """Inference execution of ``BasicUpdateBlock`` with every convolution on the split-fp16 matrix-core kernel
    (``oflow_conv_s32``: operands as fp16 hi + lo pairs, three MFMAs per product, fp32 accumulation — fp32-level
    accuracy, see csrc/conv_s32.hip) and every elementwise stage fused into a convolution epilogue.

    Activations live in S32 buffers (split-fp16 NHWC by 32-channel groups, include/oflow.h), laid out so that no
    concatenation is ever copied (`update.py:93, 96, 100, 103, 127, 155`):
      hx  = [h | motion(126) | flow(2)]   (GRU input of the z, r gates)     8 groups
      rhx = [r*h | motion | flow]          (GRU input of the candidate)      8 groups
      cf  = [relu(convc2) (192) | relu(convf2) (64)]  (input of the motion conv)  8 groups
    h is also kept in fp32 ([P, 128]) so that the blend h = (1-z)h + zq (`update.py:97`) runs in fp32.
    The GRU input is x = [inp | motion] (`update.py:153-154`) and inp, cnet's context half (`raft.py:115-118`), never
    changes across iterations: its share of every z / r / q pre-activation, W_inp * inp + bias, is computed once per
    forward for both passes (fp32 [P, 384] per pass: z | r | q) and added in the GRU epilogues, so the per-iteration
    convolutions contract [h | motion | flow] only (K: 12 -> 8 groups).
    Per iteration: the lookup fused into convc1 (oflow_corr_lookup_convc1_s32: the lookup volume is never written;
    otherwise lookup -> fp32 NHWC rows -> convc1), flow_prep -> flow channels + convf1's 7x7 patch matrix, then
    convc2, convf1 (1x1 over the patches), convf2, conv (-> hx, rhx), [z|r] (-> z, r*h -> rhx),
    q (-> h, hx) for the 1x5 and the 5x1 half, flow head conv1, conv2 (coords1 += delta in its epilogue), and at the
    last iteration the mask head (1x1 conv 256 -> 576 with the x0.25 in its epilogue, fp32 NCHW).
    """

    def __init__(self, block: BasicUpdateBlock, cnet_out: Tensor, hdim: int, side_slot: int = 0,
                 fuse_c1: bool = True, flow_head_pixels: Optional[int] = None, side_owner=None) -> None:
        b, c, h, w = cnet_out.shape
        enc, gru = block.encoder, block.gru
        cdim = c - hdim
        if (hdim, cdim, enc.conv.out_channels, gru.convz1.in_channels) != (128, 128, 126, 384):
            raise RuntimeError("SplitUpdate: supports the RAFT (large) update block only")
        dev = cnet_out.device
        self.block, self.shape = block, (b, h, w)
        # the flow head's output conv: the fp32-FMA kernel or the split conv (not bit-identical to each other), chosen
        # from the pixel count of the WHOLE forward's batch so that pair lanes give the single-lane results bit for bit
        px = b * h * w if flow_head_pixels is None else int(flow_head_pixels)
        self.flow_head_fma = px < _native.FLOW_HEAD2_MAX_PIXELS
        self.f1_from_flow = px >= CONVF1_FROM_FLOW_MIN_PIXELS
        # split-K scratch, one per runner (the calls sharing it are ordered on this runner's stream)
        self.ks = _native.KSplit(b, h, w, dev) if KSPLIT_LAYERS and px >= KSPLIT_MIN_PIXELS else None
        self.ks_mo = self.ks if "mo" in KSPLIT_LAYERS else None
        self.ks_q = self.ks if "q" in KSPLIT_LAYERS else None
        S = _native.s32_empty
        self.hx = S(b, h, w, 8, dev)
        self.rhx = S(b, h, w, 8, dev)
        levels, radius = block.corr_levels, block.corr_radius
        self.corr_ch = levels * (2 * radius + 1) ** 2  # convc1's input: fp32 NHWC lookup rows in the reference order
        self.corr_f32 = None  # [B*H*W, corr_ch], allocated on first use
        self.c1 = S(b, h, w, 8, dev)
        self.cf = S(b, h, w, 8, dev)
        self.pm = None if self.f1_from_flow else S(b, h, w, 4, dev)  # convf1's patch matrix (small grids only)
        self.f1 = S(b, h, w, 4, dev)
        self.fh = S(b, h, w, 8, dev)
        self.fh2y = None  # (B, 18, H, W) per-tap products of the flow head's output conv (flow_head_mode "col2im")
        self.flow_head_mode = getattr(block, "flow_head_mode", FLOW_HEAD_MODE)
        self.hm = torch.empty((b * h * w, hdim), device=dev, dtype=torch.float32)
        self.z = torch.empty_like(self.hm)
        V = _native.S32Slice
        _native.pack_s32(cnet_out[:, :hdim], "tanh", V(self.hx, 0, 4), nhwc=self.hm)  # raft.py:117
        inp = S(b, h, w, 4, dev)
        _native.pack_s32(cnet_out[:, hdim:], "relu", V(inp))  # raft.py:118
        self.w = self._weights(block)
        # the GRU's loop-invariant context term of both passes: [z | r | q] pre-activations of inp + bias
        self.gx = []
        for tag in ("1", "2"):
            gx = torch.empty((b * h * w, 3 * hdim), device=dev, dtype=torch.float32)
            _native.conv_s32(V(inp), self.w["inp" + tag], 128, nhwc=gx)
            self.gx.append(gx)
        self.fuse_c1 = fuse_c1 and "c1L" in self.w
        # side stream for the motion encoder's flow branch (one per device, reused across forwards)
        self.streams = getattr(block, "split_streams", True)
        # (keyed by the stream this runner's update() runs on: ``side_owner``, default the current stream)
        self.side_stream = None
        if self.streams:
            if side_owner is None:
                self.side_stream = _side_stream(dev, side_slot)
            else:
                with torch.cuda.stream(side_owner):
                    self.side_stream = _side_stream(dev, side_slot)

    @staticmethod
    def _weights(block: BasicUpdateBlock):
        return cached_pack(block, _weights_key(block), lambda: SplitUpdate._pack(block))

    @staticmethod
    def _pack(block: BasicUpdateBlock):
        enc, gru, fh = block.encoder, block.gru, block.flow_head
        CW = _native.ConvWeights
        w = {
            "c1": CW(enc.convc1.weight, enc.convc1.bias, 256),
            "c2": CW(enc.convc2.weight, enc.convc2.bias, 192),
            "f1": CW(enc.convf1.weight, enc.convf1.bias, 128, patches=True),
            "f2": CW(enc.convf2.weight, enc.convf2.bias, 64),
            "mo": CW(enc.conv.weight, enc.conv.bias, 128),
            "fh1": CW(fh.conv1.weight, fh.conv1.bias, 256),
            "fh2": CW(fh.conv2.weight, fh.conv2.bias, 32),
            # the output conv as a 1x1 conv C -> 18 (channel (ky*3+kx)*2 + c: tap (ky, kx)'s share of output c, taken at
            # the input pixel) + oflow_flow_head_col2im_f32, which gathers the 9 taps and adds the bias into coords1
            "fh2T": CW(fh.conv2.weight.detach().float().permute(2, 3, 0, 1).reshape(18, -1, 1, 1), None, 32),
            "fh2_bias": fh.conv2.bias.detach().float().contiguous(),
            # small grids: the 2-channel output conv as fp32 FMAs (oflow_flow_head2_s32) on the conv's own weights
            "fh2_f32": (fh.conv2.weight.detach().float().contiguous(), fh.conv2.bias.detach().float().contiguous()),
            # large grids: the same as fp32 FMAs on an LDS-staged halo (oflow_flow_head2_tiled_s32), repacked weights
            "fh2_tiled": (_native.flow_head2_tiled_weights(fh.conv2.weight), fh.conv2.bias.detach().float().contiguous()),
            "m1": CW(block.mask[0].weight, block.mask[0].bias, 256),
            "m2": CW(block.mask[2].weight, block.mask[2].bias, 576),
        }
        if block.corr_radius in (3, 4):  # the lookup fused into convc1 (corr_convc1.hip): weights regrouped per level
            w["c1L"] = _native.convc1_level_weights(enc.convc1, block.corr_levels, block.corr_radius)
        for tag in ("1", "2"):
            # GRU input channels (update.py:93-103): [h 0..127 | inp 128..255 | motion 256..381 | flow 382, 383]; the
            # per-iteration convs take [h | motion | flow] (no bias), the hoisted one inp with the z | r | q biases
            cz, cr, cq = (getattr(gru, f"conv{g}{tag}") for g in "zrq")
            hmf = lambda wt: torch.cat([wt[:, :128], wt[:, 256:]], dim=1)
            w["zr" + tag] = CW(hmf(torch.cat([cz.weight, cr.weight])), None, 256)
            w["q" + tag] = CW(hmf(cq.weight), None, 128)
            w["inp" + tag] = CW(torch.cat([cz.weight, cr.weight, cq.weight])[:, 128:256],
                                torch.cat([cz.bias, cr.bias, cq.bias]), 384)
        return w

    def step(self, corr_fn, coords1: Tensor, need_mask: bool, mask_out: Optional[Tensor] = None) -> Optional[Tensor]:
        """One update (`update.py:150-161` + `raft.py:128-133`): coords1 is advanced IN PLACE by delta_flow.
        Returns 0.25 * mask (B, 576, H, W) fp32 when ``need_mask`` (written into ``mask_out`` if given), else None."""
        return self.update(self.lookup(corr_fn, coords1), coords1, need_mask, mask_out)

    def lookup_rows(self, coords1: Tensor) -> Tensor:
        """The fp32 NHWC lookup buffer [B*H*W, L*(2r+1)^2] (allocated on first use)."""
        if self.corr_f32 is None:
            b, h, wd = self.shape
            self.corr_f32 = torch.empty((b * h * wd, self.corr_ch), device=coords1.device, dtype=torch.float32)
        return self.corr_f32

    def fusable(self, corr_fn) -> bool:
        """Whether convc1 takes its input straight from ``corr_fn``'s tiled pyramid (oflow_corr_lookup_convc1_s32)."""
        return self.fuse_c1 and getattr(corr_fn, "_tiled", None) is not None and corr_fn.radius in (3, 4)

    def lookup(self, corr_fn, coords1: Tensor):
        """The correlation lookup as convc1's input (`raft.py:128`): the tiled pyramid itself when the lookup runs
        inside convc1 (``FusedLookup``), else fp32 NHWC rows split while convc1 stages them."""
        if self.fusable(corr_fn):
            return FusedLookup(corr_fn._tiled, coords1, corr_fn.radius)
        b, h, wd = self.shape
        corr_fn.lookup_nhwc(coords1, self.lookup_rows(coords1))
        return _native.F32In(self.corr_f32, b, h, wd)

    def _convc1(self, corr_in) -> None:
        """relu(convc1(corr)) -> c1 (`update.py:120`)."""
        if isinstance(corr_in, FusedLookup):
            _native.corr_lookup_convc1(corr_in.pyr, corr_in.coords, corr_in.radius, self.w["c1L"], _native.S32Slice(self.c1))
        else:
            _native.conv_s32(corr_in, self.w["c1"], 128, "relu", y0=_native.S32Slice(self.c1))

    def update(self, corr_in, coords1: Tensor, need_mask: bool, mask_out: Optional[Tensor] = None) -> Optional[Tensor]:
        """Everything of one update after the lookup; ``corr_in`` is convc1's input (F32In)."""
        V, conv, w = _native.S32Slice, _native.conv_s32, self.w
        b, h, wd = self.shape
        # The motion encoder's two branches are independent (update.py:116-121): the flow branch (flow prep, convf1,
        # convf2) runs on a side stream beside the correlation branch (convc1, convc2), both MFMA-latency bound, and
        # joins before the motion conv. The side stream starts after the lookup, which thus runs alone (its bench
        # timing stays uncontended). Buffers are persistent and disjoint (cf groups 6-7 vs 0-5; the GRU inputs' flow
        # group is read again only after the join).
        main = torch.cuda.current_stream(coords1.device)
        side = self.side_stream if self.streams else None
        bns = CONV_BN_SIDE if side is not None else CONV_BN  # (channel blocks: see CONV_BN)
        f1_in = V(self.pm) if self.pm is not None else _native.FlowIn(coords1)
        if side is not None:
            side.wait_stream(main)
            with torch.cuda.stream(side):
                _native.flow_prep(coords1, self.pm, (V(self.hx), 254), (V(self.rhx), 254))
                conv(f1_in, w["f1"], bns["f1"], "relu", y0=V(self.f1))
                conv(V(self.f1), w["f2"], bns["f2"], "relu", y0=V(self.cf, 6, 2))
            self._convc1(corr_in)
            conv(V(self.c1), w["c2"], bns["c2"], "relu", y0=V(self.cf, 0, 6))
            main.wait_stream(side)
        else:
            _native.flow_prep(coords1, self.pm, (V(self.hx), 254), (V(self.rhx), 254))
            self._convc1(corr_in)
            conv(V(self.c1), w["c2"], bns["c2"], "relu", y0=V(self.cf, 0, 6))
            conv(f1_in, w["f1"], bns["f1"], "relu", y0=V(self.f1))
            conv(V(self.f1), w["f2"], bns["f2"], "relu", y0=V(self.cf, 6, 2))
        conv(V(self.cf), w["mo"], bns["mo"], "relu", y0=V(self.hx, 4, 4), y1=V(self.rhx, 4, 4), ksplit=self.ks_mo)
        for tag, gx in zip(("1", "2"), self.gx):
            conv(V(self.hx), w["zr" + tag], bns["gru"], epilogue=1, y0=V(self.rhx, 0, 4), gru_h=self.hm, gru_z=self.z,
                 addend=gx[:, :256])
            conv(V(self.rhx), w["q" + tag], bns["gru"], epilogue=2, y0=V(self.hx, 0, 4), gru_h=self.hm, gru_z=self.z,
                 addend=gx[:, 256:], ksplit=self.ks_q)
        net = V(self.hx, 0, 4)
        conv(net, w["fh1"], bns["fh1"], "relu", y0=V(self.fh))
        if self.flow_head_fma and coords1.is_contiguous():
            _native.flow_head2(V(self.fh), *w["fh2_f32"], coords1)  # coords1 += conv2(.) (raft.py:133)
        elif self.flow_head_mode == "tiled" and coords1.is_contiguous():
            _native.flow_head2_tiled(V(self.fh), *w["fh2_tiled"], coords1)  # coords1 += conv2(.) (raft.py:133)
        elif self.flow_head_mode == "col2im" and coords1.is_contiguous():
            if self.fh2y is None:
                self.fh2y = torch.empty((b, 18, h, wd), device=coords1.device, dtype=torch.float32)
            conv(V(self.fh), w["fh2T"], 32, f32=self.fh2y)
            _native.flow_head_col2im(self.fh2y, w["fh2_bias"], coords1)  # coords1 += conv2(.) (raft.py:133)
        else:
            conv(V(self.fh), w["fh2"], 32, f32=coords1, f32_accumulate=True)
        if not need_mask:
            return None
        mask = mask_out if mask_out is not None else torch.empty((b, 576, h, wd), device=coords1.device, dtype=torch.float32)
        conv(net, w["m1"], 128, "relu", y0=V(self.fh))
        conv(V(self.fh), w["m2"], 64, out_scale=0.25, f32=mask)
        return mask
