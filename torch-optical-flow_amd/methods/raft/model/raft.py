"""RAFT inference model (reference: methods/raft/model/raft.py:21-147), MI355X-native correlation path.

Same constructor arguments, ``hparams`` attribute, sub-modules and ``state_dict`` keys as the reference's
LightningModule, so its checkpoints load unchanged; the training loop (`raft.py:149-260`: loss, optimizers,
W&B logging) is out of scope. ``forward`` keeps the reference's semantics and return
values; three output-identical changes remove host work from the loop:
  * the correlation pyramid and every lookup run on the gfx950 kernels (``model.corr.CorrBlock``);
    ``alternate_corr=True`` (an addition, default off) swaps in the volume-free fp16 ``AlternateCorrBlock``
    for large frames;
  * coordinate grids are built on the device (no CPU build + H2D copy, `raft.py:68-69`);
  * with ``test_mode=True`` only the last iteration's convex upsampling is computed — the reference computes
    all ``iters`` and returns only the last (Q11, `raft.py:136-145`);
  * without autograd on the GPU the encoders run through ``SplitEncoder`` (split-fp16 convolutions, fp64-merged
    instance-norm statistics, folded eval batch norm; ``encoder_impl = "module"`` keeps the nn.Modules) and the
    update block runs through ``SplitUpdate``: every convolution on the
    split-fp16 matrix-core kernel (fp32-level accuracy) with the GRU gates, activations, concatenations and the
    ``coords1 += delta_flow`` update fused into convolution epilogues (``update_impl = "fused"`` selects the
    MIOpen-based ``FusedUpdate`` instead); in test mode the mask head (two convolutions feeding only the
    upsampling) runs at the last iteration only.
"""
from __future__ import annotations

import os
from typing import Any, Dict, List, Optional, Tuple, Union

import torch
import torch.nn as nn
import torch.nn.functional as F
from torch import Tensor

from optical_flow import _native

from .corr import AlternateCorrBlock, CorrBlock
from .extractor import BasicEncoder, SplitEncoder
from .update import BasicUpdateBlock, FusedUpdate, SplitUpdate, _side_stream, capture_active
from .utils import coords_grid, upflow8

# RAFT.forward's input scaling (raft.py:104-105) through oflow_normalize_images_f32 on GPU inference: one kernel for
# both frames, bit-identical to the reference's CPU arithmetic (ATen on the GPU divides by multiplying with fl(1/255),
# 1 ulp off for ~74 % of values); in-process step 18.56 -> 18.48 ms (profiles/r04/s35_ab.log). False: the ATen form.
NATIVE_NORMALIZE = True
# the pair lanes' SplitUpdate state (cnet output packed into the GRU state, the hoisted context terms) built on the cnet
# stream right after cnet, beside fnet's tail and the correlation pyramid, instead of on the lanes after the pyramid
EARLY_LANE_INIT = True


class HParams(dict):
    """Attribute access to the constructor arguments (Lightning's ``self.hparams`` as used in `raft.py`)."""

    def __getattr__(self, key: str) -> Any:
        try:
            return self[key]
        except KeyError as e:
            raise AttributeError(key) from e


def strip_module(state_dict: Dict[str, Tensor]) -> Dict[str, Tensor]:
    """Drop the ``module.`` prefix of DataParallel checkpoints (reference `pretrained/convert.py:4-11`)."""
    return {(k[7:] if k.startswith("module.") else k): v for k, v in state_dict.items()}


def _drop_weight_cache(module: nn.Module, _incompatible) -> None:
    module.__dict__.pop("_split_weights", None)


class RAFT(nn.Module):
    def __init__(
        self,
        hidden_dim: int = 128,
        context_dim: int = 128,
        corr_levels: int = 4,
        corr_radius: int = 4,
        iters: int = 12,
        iters_val: int = 24,
        gamma: float = 0.8,
        dropout: float = 0.0,
        lr: float = 0.00002,
        wdecay: float = 0.00005,
        epsilon: float = 1e-8,
        alternate_corr: bool = False,
    ) -> None:
        super().__init__()
        self.hparams = HParams(
            hidden_dim=hidden_dim,
            context_dim=context_dim,
            corr_levels=corr_levels,
            corr_radius=corr_radius,
            iters=iters,
            iters_val=iters_val,
            gamma=gamma,
            dropout=dropout,
            lr=lr,
            wdecay=wdecay,
            epsilon=epsilon,
            alternate_corr=alternate_corr,
        )
        self.fnet = BasicEncoder(output_dim=256, norm_fn="instance", dropout=dropout)
        self.cnet = BasicEncoder(output_dim=hidden_dim + context_dim, norm_fn="batch", dropout=dropout)
        self.update_block = BasicUpdateBlock(corr_levels=corr_levels, corr_radius=corr_radius, hidden_dim=hidden_dim)
        # plain attributes (not hparams): how GPU inference runs the update block. "split": split-fp16 matrix-core
        # convolutions with fused epilogues (SplitUpdate, default); "fused": MIOpen fp32 convolutions + fused
        # elementwise kernels (FusedUpdate); "module": the nn.Module as written. fused_update=False forces "module".
        self.update_impl = "split"
        self.fused_update = True
        # "split": encoders on the split-fp16 kernels (SplitEncoder) in GPU inference; "module": nn.Module (MIOpen)
        self.encoder_impl = "split"
        self.encoder_streams = True  # cnet beside fnet + the corr pyramid (inference, split encoders)
        self.fnet_streams = True  # with encoder_streams: fnet's image0 and image1 halves on two streams
        # split update loop over >= 2 pairs (CorrBlock): the pairs' two halves run on two streams so that one half's
        # convolutions fill the CUs the other half's leave idle at a wave tail. pair_lookup "joined": one full-batch
        # lookup per iteration on the main stream (both halves joined around it); "lane": each half looks up its own.
        self.pair_lanes = 2
        self.pair_lookup = "joined"
        # lookup fused into convc1 (csrc/corr_convc1.hip; CorrBlock, radius 3 / 4): each lane runs
        # relu(convc1(lookup)) as one kernel and the lookup volume never reaches HBM (pair_lookup then does not apply)
        self.lookup_fusion = True
        # with the split encoders, fnet writes its features as S32 rows and the pyramid is built from split-fp16
        # products (oflow_corr_pyramid_tiled_s32); False: fp32 features and the fp32-MFMA pyramid
        self.split_corr = True
        # split encoders: the stem convolution builds its 7x7 patch operand from the image tile by tile
        # (OFLOW_IN_IMG7S2) instead of reading a patch matrix written beforehand (fnet's image0 rows shared with cnet)
        self.stem_from_image = True
        # the split-fp16 range guard (csrc: a sticky device flag set when an operand's hi half overflows fp16). After
        # each GPU inference forward the flag is read and cleared in one device-side exchange on the forward's stream
        # (``_native.RangeSnapshot``: that forward's own status, copied to pinned memory behind an event).
        # "deferred" (default): no host sync in the forward; the snapshot is ``last_range_snapshot`` (callers that
        # consume the output asynchronously check it before using it, as predict.py's writer does), a later forward
        # raises once the GPU is past an overflowing one, and check_range() waits and raises. "sync": the forward
        # waits for its snapshot and raises (one host sync per forward: -2.5 % on the 8-pair bench step,
        # profiles/r04/s1_bench*.log). "off": never read (the flag then stays set until another model reads it).
        self.range_guard = "deferred"
        self._range_pending = []  # deferred snapshots not yet checked, in issue order
        self.last_range_snapshot = None
        # the split paths cache packed fp16 hi/lo weights keyed by (storage, version); parameters created under
        # torch.inference_mode() have no version counter, so loading new weights in place drops the caches
        for m in (self.fnet, self.cnet, self.update_block):
            m.register_load_state_dict_post_hook(_drop_weight_cache)

    def invalidate_weight_caches(self) -> None:
        """Drop the packed-weight caches of the split kernels (call after editing parameters in place under
        torch.inference_mode(); load_state_dict does it by itself)."""
        for m in (self.fnet, self.cnet, self.update_block):
            _drop_weight_cache(m, None)

    # -- checkpoints -------------------------------------------------------------------------------------
    @classmethod
    def load_from_checkpoint(cls, checkpoint_path: Union[str, os.PathLike], map_location=None, **kwargs) -> "RAFT":
        """Load a Lightning ``.ckpt`` (``state_dict`` + ``hyper_parameters``) or an official ``.pth``
        (``module.``-prefixed keys) with ``torch.load(weights_only=True)``."""
        ckpt = torch.load(checkpoint_path, map_location=map_location or "cpu", weights_only=True)
        hp = {}
        if isinstance(ckpt, dict) and "state_dict" in ckpt:
            hp = dict(ckpt.get("hyper_parameters", {}) or {})
            sd = ckpt["state_dict"]
        else:
            sd = ckpt
        hp.update(kwargs)
        model = cls(**{k: v for k, v in hp.items() if k in cls.__init__.__code__.co_varnames})
        sd = {k: v for k, v in strip_module(sd).items() if not k.startswith(("epe_", "f1_"))}
        model.load_state_dict(sd)
        return model

    def freeze_bn(self) -> None:
        for m in self.modules():
            if isinstance(m, nn.BatchNorm2d):
                m.eval()

    # -- forward -----------------------------------------------------------------------------------------
    @staticmethod
    def initialize_flow(img: Tensor) -> Tuple[Tensor, Tensor]:
        """coords0 = coords1 = pixel grid at 1/8 resolution; flow = coords1 - coords0 (`raft.py:64-71`)."""
        n, _, h, w = img.shape
        coords0 = coords_grid(n, h // 8, w // 8, device=img.device)
        return coords0, coords0.clone()

    @staticmethod
    def upsample_flow(flow: Tensor, mask: Tensor) -> Tensor:
        """[H/8, W/8, 2] -> [H, W, 2] by a softmax-weighted 3x3 convex combination (`raft.py:73-85`)."""
        if flow.is_cuda and not (torch.is_grad_enabled() and (flow.requires_grad or mask.requires_grad)):
            return _native.convex_upsample(flow, mask)  # one fused HIP kernel (csrc/upsample.hip)
        n, _, h, w = flow.shape
        mask = torch.softmax(mask.view(n, 1, 9, 8, 8, h, w), dim=2)
        up_flow = F.unfold(8 * flow, [3, 3], padding=1).view(n, 2, 9, 1, 1, h, w)
        up_flow = torch.sum(mask * up_flow, dim=2).permute(0, 1, 4, 2, 5, 3)
        return up_flow.reshape(n, 2, 8 * h, 8 * w)

    def _lane_cuts(self, b: int):
        n = min(self.pair_lanes, b)
        edges = [(b * i) // n for i in range(n + 1)]
        return list(zip(edges[:-1], edges[1:]))

    def _lane_runners(self, cnet_out: Tensor, hdim: int, lanes, on=None) -> list:
        """One SplitUpdate per lane (its buffers, the cnet output packed into the GRU state, the loop-invariant context
        terms), built on stream ``on`` (default: each lane's own stream)."""
        runners = []
        for i, ((b0, b1), st) in enumerate(zip(self._lane_cuts(cnet_out.shape[0]), lanes)):
            with torch.cuda.stream(on if on is not None else st):
                slot = 0 if i == 0 else 200 + i
                runners.append(SplitUpdate(self.update_block, cnet_out[b0:b1], hdim, side_slot=slot, fuse_c1=self.lookup_fusion,
                                           flow_head_pixels=cnet_out.shape[0] * cnet_out.shape[2] * cnet_out.shape[3],
                                           side_owner=st))
        return runners

    def _lanes_for(self, dev, b: int):
        main = torch.cuda.current_stream(dev)
        return [main] + [_side_stream(dev, 100 + i) for i in range(1, min(self.pair_lanes, b))]

    def _split_update_lanes(self, corr_fn, cnet_out: Tensor, coords0: Tensor, coords1: Tensor, iters: int, hdim: int,
                            test_mode: bool, runners=None) -> List[Tensor]:
        """The split update loop with the pairs in ``pair_lanes`` parts, each on its own stream (lane) with its own side stream;
        coords1 is advanced in place. Per-pixel results are those of the single-lane loop bit for bit (no reduction
        crosses pairs). Returns the upsampled flows (test mode: the last one only). ``runners``: the lanes' SplitUpdates
        when already built (on the cnet stream, beside the correlation pyramid; the current stream has waited for it)."""
        b = cnet_out.shape[0]
        dev = cnet_out.device
        cuts = self._lane_cuts(b)
        main = torch.cuda.current_stream(dev)
        lanes = self._lanes_for(dev, b)
        # the packed weights (built on first use, by kernels on this stream) must exist before the lanes fork: the
        # lanes read them with no later join when the lookup is not joined (fused into convc1, or pair_lookup "lane")
        SplitUpdate._weights(self.update_block)
        # lane_init_on_main: the lanes' buffers are allocated (and their loop-invariant context terms computed) on the
        # main stream before the fork, so that no lane allocates from its own stream
        init_main = getattr(self, "lane_init_on_main", False) or runners is not None
        if not init_main:
            for st in lanes[1:]:
                st.wait_stream(main)
        if runners is None:
            runners = self._lane_runners(cnet_out, hdim, lanes, on=main if init_main else None)
        if init_main:
            for st in lanes[1:]:
                st.wait_stream(main)
        joined = self.pair_lookup == "joined" and not runners[0].fusable(corr_fn)
        hw = cnet_out.shape[2] * cnet_out.shape[3]
        if joined:
            rows = torch.empty((b * hw, runners[0].corr_ch), device=dev, dtype=torch.float32)
            h, w = cnet_out.shape[2:]
            ins = [_native.F32In(rows[b0 * hw : b1 * hw], b1 - b0, h, w) for b0, b1 in cuts]
        else:
            parts = [corr_fn.batch_slice(b0, b1) for b0, b1 in cuts]
        outs = []
        for itr in range(iters):
            last = itr == iters - 1
            need = not test_mode or last
            mask = torch.empty((b, 576, *cnet_out.shape[2:]), device=dev, dtype=torch.float32) if need else None
            if joined:
                for st in lanes[1:]:
                    main.wait_stream(st)
                corr_fn.lookup_nhwc(coords1, rows)
            if joined or need:  # (need: the mask block may still be in use by earlier main-stream work)
                for st in lanes[1:]:
                    st.wait_stream(main)
            for i, ((b0, b1), st) in enumerate(zip(cuts, lanes)):
                with torch.cuda.stream(st):
                    c1 = coords1[b0:b1]
                    corr_in = ins[i] if joined else runners[i].lookup(parts[i], c1)
                    runners[i].update(corr_in, c1, need, mask_out=mask[b0:b1] if need else None)
            if need:
                for st in lanes[1:]:
                    main.wait_stream(st)
                outs.append(self.upsample_flow(coords1 - coords0, mask))
        for st in lanes[1:]:
            main.wait_stream(st)
        return outs

    def check_range(self, device=None) -> None:
        """Raise if a split-fp16 operand overflowed in any forward since the last check (waits for those forwards; with
        ``device`` also reads the flag after every stream of it, e.g. forwards of range_guard "off")."""
        pend, self._range_pending = self._range_pending, []
        bad = False
        for snap in pend:
            bad |= snap.overflowed()
        if bad:
            raise RuntimeError(f"RAFT forward: in an earlier forward {_native.RANGE_ERROR}")
        if device is not None:
            _native.range_flag_raise_if_set(device, all_streams=True)

    def forward(
        self,
        image0: Tensor,
        image1: Tensor,
        iters: int = 12,
        flow_init: Optional[Tensor] = None,
        upsample: bool = True,
        test_mode: bool = False,
    ) -> Union[Tensor, Tuple[Tensor, Tensor], List[Tensor]]:
        """Estimate optical flow between pairs of frames (`raft.py:87-147`). Images (B, 3, H, W) in [0, 255]
        with H, W divisible by 8 (use ``InputPadder``). Returns ``(coords1 - coords0, flow_up)`` in test mode,
        else the list of ``iters`` upsampled predictions. On the GPU in inference the split-fp16 range guard
        (``range_guard``) reports an operand that left the fp16 range with RuntimeError: "sync" raises from this
        forward; "deferred" (default) does not wait -- this forward's status is ``last_range_snapshot``
        (``.overflowed()`` waits for it), and a later forward or ``check_range()`` raises for it."""
        guard = self.range_guard in ("sync", "deferred") and image0.is_cuda and not torch.is_grad_enabled()
        capturing = image0.is_cuda and capture_active(image0.device)
        if guard and not capturing:
            self._range_before(image0.device)
        out = self._forward(image0, image1, iters, flow_init, test_mode)
        if guard and not capturing:
            self._range_after(image0.device)
        return out

    def _range_before(self, dev) -> None:
        """Register the device's range flag; in deferred mode raise for an earlier forward the GPU has finished."""
        _native.range_flag(dev)  # registered before the first kernel that may set it
        if self.range_guard != "deferred":
            return
        bad = False
        while self._range_pending and self._range_pending[0].done():
            bad |= self._range_pending.pop(0).overflowed()
        if bad:
            raise RuntimeError(f"RAFT forward: in an earlier forward {_native.RANGE_ERROR}")

    def _range_after(self, dev) -> None:
        """After a forward's kernels are enqueued: its snapshot (exchange + copy on the current stream); "sync" waits for
        it and raises."""
        snap = _native.RangeSnapshot(torch.device(dev)).take()  # (a new one per forward: callers may hold the last)
        self.last_range_snapshot = snap
        if self.range_guard == "sync":
            if snap.overflowed():
                raise RuntimeError(f"RAFT forward: {_native.RANGE_ERROR}")
        else:
            self._range_pending.append(snap)

    def _forward(self, image0: Tensor, image1: Tensor, iters: int, flow_init: Optional[Tensor], test_mode: bool):
        if (NATIVE_NORMALIZE and image0.is_cuda and image1.is_cuda and image0.dtype == image1.dtype == torch.float32
                and image0.shape == image1.shape
                and not (torch.is_grad_enabled() and (image0.requires_grad or image1.requires_grad))):
            # raft.py:104-105 as one kernel for both frames (ATen: three launches per frame)
            image0, image1 = _native.normalize_images(image0, image1)
        else:  # CPU tensors, or frames that need gradients (autograd through the elementwise form)
            image0 = (2 * (image0 / 255.0) - 1.0).contiguous()
            image1 = (2 * (image1 / 255.0) - 1.0).contiguous()
        hdim, cdim = self.hparams.hidden_dim, self.hparams.context_dim

        # the split encoders implement the inference forward: fnet in train mode with dropout > 0 applies Dropout2d in
        # the reference (extractor.py BasicEncoder.forward), so it then runs as the module (cnet likewise: batch norm)
        split_enc = (
            image0.is_cuda
            and not torch.is_grad_enabled()
            and self.encoder_impl == "split"
            and (not self.fnet.training or self.fnet.dropout is None)
        )
        fnet = SplitEncoder(self.fnet) if split_enc else self.fnet
        cnet = SplitEncoder(self.cnet) if split_enc and not self.cnet.training else self.cnet
        block = AlternateCorrBlock if self.hparams.get("alternate_corr", False) else CorrBlock
        pre_runners = None
        if split_enc and isinstance(cnet, SplitEncoder):
            # image0's stem patches are the first rows of fnet's (raft.py:109, 115 feed both the same image0); cnet
            # runs on a side stream beside fnet and the correlation pyramid, joined before the update loop
            main = torch.cuda.current_stream(image0.device)
            side = _side_stream(image0.device) if self.encoder_streams else None
            nb = image0.shape[0]
            side2 = (_side_stream(image0.device, 1) if side is not None and self.fnet_streams
                     and block is CorrBlock and self.split_corr else None)
            sfi = self.stem_from_image
            if side2 is not None:
                # fnet's two images on two streams (instance norm is per image: the same values as one batch), so
                # three 8-image encoders share the chip and finish together
                side2.wait_stream(main)
                with torch.cuda.stream(side2):
                    f2s = fnet(image1, split_out=True, stem_from_image=sfi)
                patches = None if sfi else fnet.stem_patches(image0)
            else:
                patches = None if sfi else fnet.stem_patches(torch.cat([image0, image1], dim=0))
            cpatches = None if patches is None else patches[:nb]
            early = (EARLY_LANE_INIT and side is not None and self.fused_update and self.update_impl == "split"
                     and self.pair_lanes > 1 and nb > 1 and block is CorrBlock and self.split_corr)
            lanes = self._lanes_for(image0.device, nb) if early else None  # (main = the current stream, not cnet's)
            if side is not None:
                side.wait_stream(main)
                with torch.cuda.stream(side):
                    cnet_out = cnet(image0, patches=cpatches, stem_from_image=sfi)
                    if early:
                        # the lanes' GRU state and context terms depend on cnet only: built here, beside fnet's tail
                        # and the correlation pyramid, instead of after the pyramid on the lanes
                        SplitUpdate._weights(self.update_block)
                        pre_runners = self._lane_runners(cnet_out, hdim, lanes, on=side)
            if block is CorrBlock and self.split_corr:
                # features as S32 rows straight from fnet's head conv -> split-fp16 pyramid (no fp32 fmaps)
                if side2 is not None:
                    f1s = fnet(image0, patches=patches, split_out=True, stem_from_image=sfi)
                    main.wait_stream(side2)
                else:
                    f1s, f2s = fnet([image0, image1], patches=patches, split_out=True, stem_from_image=sfi)
                corr_fn = CorrBlock.from_split_features(f1s, f2s, radius=self.hparams.corr_radius)
            else:
                fmap1, fmap2 = fnet([image0, image1], patches=patches, stem_from_image=sfi)
                corr_fn = block(fmap1.float(), fmap2.float(), radius=self.hparams.corr_radius)
            if side is not None:
                main.wait_stream(side)
            else:
                cnet_out = cnet(image0, patches=cpatches, stem_from_image=sfi)
        else:
            fmap1, fmap2 = fnet([image0, image1])
            corr_fn = block(fmap1.float(), fmap2.float(), radius=self.hparams.corr_radius)
            cnet_out = cnet(image0)
        coords0, coords1 = self.initialize_flow(image0)
        if flow_init is not None:
            coords1 = coords1 + flow_init

        gpu_inference = cnet_out.is_cuda and not torch.is_grad_enabled() and self.fused_update
        impl = self.update_impl if gpu_inference else "module"
        flow_predictions = []
        flow_up = None
        if impl == "split" and self.pair_lanes > 1 and cnet_out.shape[0] > 1 and hasattr(corr_fn, "lookup_nhwc"):
            coords1 = coords1.contiguous()
            flow_predictions = self._split_update_lanes(corr_fn, cnet_out, coords0, coords1, iters, hdim, test_mode,
                                                        runners=pre_runners)
            if test_mode:
                return coords1 - coords0, flow_predictions[-1]
            return flow_predictions
        if impl == "split":
            # coords1 is advanced in place by the flow head's epilogue (raft.py:133)
            runner = SplitUpdate(self.update_block, cnet_out, hdim, fuse_c1=self.lookup_fusion)
            coords1 = coords1.contiguous()
            for itr in range(iters):
                last = itr == iters - 1
                up_mask = runner.step(corr_fn, coords1, need_mask=not test_mode or last)
                if test_mode and not last:
                    continue  # Q11: intermediate upsamplings are never returned in test mode
                flow_up = self.upsample_flow(coords1 - coords0, up_mask)
                flow_predictions.append(flow_up)
            if test_mode:
                return coords1 - coords0, flow_up
            return flow_predictions

        net, inp = torch.split(cnet_out, [hdim, cdim], dim=1)
        net = torch.tanh(net)
        inp = torch.relu(inp)
        runner = FusedUpdate(self.update_block, net, inp) if impl == "fused" else None
        for itr in range(iters):
            coords1 = coords1.detach()
            corr = corr_fn(coords1)
            flow = coords1 - coords0
            last = itr == iters - 1
            if runner is not None:
                # Q11: in test mode only the last iteration's mask (upsampling) is ever used
                net, up_mask, delta_flow = runner.step(corr, flow, need_mask=not test_mode or last)
            else:
                net, up_mask, delta_flow = self.update_block(net, inp, corr, flow)
            coords1 = coords1 + delta_flow
            if test_mode and not last:
                continue  # Q11: intermediate upsamplings are never returned in test mode
            if up_mask is None:
                flow_up = upflow8(coords1 - coords0)
            else:
                flow_up = self.upsample_flow(coords1 - coords0, up_mask)
            flow_predictions.append(flow_up)

        if test_mode:
            return coords1 - coords0, flow_up
        return flow_predictions
