"""ctypes binding of liboflow_hip.so (C ABI declared in include/oflow.h) for torch tensors.

PyTorch supplies device memory (its caching allocator) and the current HIP stream; the arithmetic runs in the
hand-written gfx950 kernels of ``csrc/``. There is no fallback: on a tensor that is not on a ROCm GPU, or when
the library is missing, every entry point raises ``RuntimeError``.

``torch`` is imported before the library is opened so that the library's ``libamdhip64.so.7`` dependency
resolves (by SONAME) to the HIP runtime PyTorch already loaded: one runtime, one set of streams.
"""
from __future__ import annotations

import ctypes
import os
from typing import List, Optional, Sequence

import torch

from . import _ops

_LIB_PATH = os.environ.get(
    "OFLOW_LIB", os.path.join(os.path.dirname(os.path.abspath(__file__)), "_lib", "liboflow_hip.so")
)
ABI_VERSION = 1
MAX_LEVELS = 8
MAX_RADIUS = 7
# grids below this many pixels run the flow head output conv as oflow_flow_head2_s32 (fp32 FMAs), larger ones as
# oflow_conv_s32 (faster once the grid fills the chip): the threshold of the conv's small-grid tiles (conv_s32.hip)
FLOW_HEAD2_MAX_PIXELS = 16384
E_TINY = -4

INTERP = {"bilinear": 0, "nearest": 1, "bicubic": 2}
PADDING = {"zeros": 0, "border": 1, "reflection": 2}

# every symbol include/oflow.h declares (tests check the library exports them all)
SYMBOLS = (
    "oflow_abi_version",
    "oflow_status_string",
    "oflow_corr_pyramid_dims",
    "oflow_corr_pyramid_f32",
    "oflow_corr_lookup_f32",
    "oflow_corr_tiled_level_floats",
    "oflow_corr_pyramid_tiled_f32",
    "oflow_corr_lookup_tiled_f32",
    "oflow_corr_untile_f32",
    "oflow_grid_warp_f32",
    "oflow_grid_sample_f32",
    "oflow_corr_otf_prepare_f16",
    "oflow_corr_lookup_otf_f16",
    "oflow_bias_act_f32",
    "oflow_gru_reset_f32",
    "oflow_gru_blend_f32",
    "oflow_conv_s32",
    "oflow_pack_s32_f32",
    "oflow_flow_prep_s32",
    "oflow_conv_s32_ex",
    "oflow_stem_patches_s32",
    "oflow_norm_stats_finalize",
    "oflow_norm_apply_s32",
    "oflow_convex_upsample_f32",
    "oflow_conv_s32_ex2",
    "oflow_corr_lookup_tiled_nhwc_f32",
    "oflow_corr_lookup_backward_f32",
    "oflow_corr_pyramid_grad_combine_f32",
    "oflow_flow_stats_f32",
    "oflow_flow2rgb_f32",
    "oflow_flow_pack_f32",
    "oflow_corr_lookup_convc1_s32",
    "oflow_corr_pyramid_tiled_s32",
    "oflow_flow_head2_s32",
    "oflow_flow_head2_tiled_s32",
    "oflow_conv_s32_ex3",
    "oflow_conv_s32_ex4",
    "oflow_conv_s32_ex5",
    "oflow_normalize_images_f32",
    "oflow_replicate_pad_f32",
    "oflow_corr_fmap_grad_f32",
    "oflow_grid_warp_backward_f32",
    "oflow_grid_sample_backward_f32",
    "oflow_set_range_flag",
    "oflow_range_flag_exchange",
    "oflow_flow_head_col2im_f32",
    "oflow_timing_event_create",
    "oflow_timing_event_destroy",
    "oflow_timing_event_record",
    "oflow_timing_event_elapsed_ms",
)

_lib = None
_recorder = None  # optional {op name: [(start event, end event), ...]} filled around each launch
_flops = None  # optional {"exec_f16": .., "useful": .., "fma_f32": ..} accumulated per launch (bench's step roofline)


def set_flop_counter(counter):
    """Accumulate, per matrix-core launch, the f16 MFMA flops the kernels issue (3 split products; channel padding to
    32-channel groups and output-channel blocks included, pixel-tile padding not) under "exec_f16", the fp32-equivalent
    flops of the layer's real channels under "useful", and the fp32 FMA flops of the small-grid flow head under
    "fma_f32". ``counter``: a dict, or None to stop."""
    global _flops
    _flops = counter


def _count(exec_f16: int, useful: int, fma: int = 0) -> None:
    _flops["exec_f16"] = _flops.get("exec_f16", 0) + exec_f16
    _flops["useful"] = _flops.get("useful", 0) + useful
    _flops["fma_f32"] = _flops.get("fma_f32", 0) + fma


def set_event_recorder(recorder):
    """Record a HIP event pair on the launch stream around every kernel launch (bench instrumentation).
    ``recorder`` is a dict (op name -> list of (start, end) events) or None to stop. The events are
    ``torch.cuda.Event``s, or ``TimingEvent``s when the recorder holds ``"_native": True`` -- those may be recorded
    inside a stream capture (external event-record nodes: each replay of the graph re-records them)."""
    global _recorder
    _recorder = recorder


class TimingEvent:
    """A HIP timing event of liboflow_hip.so (oflow_timing_event_*): ``record(stream)`` on a capturing stream records
    it as an external event node of the graph (torch.cuda.Event refuses that on ROCm); ``elapsed_time(end)`` in ms,
    as torch.cuda.Event's."""

    __slots__ = ("ev",)

    def __init__(self):
        ev = ctypes.c_void_p()
        _check(load().oflow_timing_event_create(ctypes.byref(ev)), "timing_event_create")
        self.ev = ev

    def record(self, stream: "torch.cuda.Stream") -> None:
        # external = 1: the library asks HIP whether `stream` is capturing (a pair lane forked inside a capture is,
        # though torch.cuda.is_current_stream_capturing() does not say so on ROCm) and records a plain event if not
        _check(load().oflow_timing_event_record(self.ev, ctypes.c_void_p(stream.cuda_stream), 1), "timing_event_record")

    def elapsed_time(self, end: "TimingEvent") -> float:
        ms = ctypes.c_float()
        _check(load().oflow_timing_event_elapsed_ms(self.ev, end.ev, ctypes.byref(ms)), "timing_event_elapsed_ms")
        return float(ms.value)

    def __del__(self):
        try:
            if _lib is not None and self.ev:
                _lib.oflow_timing_event_destroy(self.ev)
        except Exception:  # noqa: BLE001 (interpreter shutdown)
            pass


# ops whose launches are bracketed by events when a recorder is set (others only if the recorder has "*": True)
_TIMED_DEFAULT = ("corr_lookup", "corr_lookup_convc1", "corr_pyramid", "corr_lookup_otf", "corr_otf_prepare", "grid_warp")


class _Timed:
    __slots__ = ("what", "stream", "ev0")

    def __init__(self, what: str, device: torch.device):
        self.what = what
        on = _recorder is not None and (what in _TIMED_DEFAULT or _recorder.get("*", False))
        self.stream = torch.cuda.current_stream(device) if on else None
        self.ev0 = None

    def __enter__(self):
        if self.stream is not None:
            self.ev0 = TimingEvent() if _recorder.get("_native") else torch.cuda.Event(enable_timing=True)
            self.ev0.record(self.stream)
        return self

    def __exit__(self, *exc):
        if self.stream is not None and exc[0] is None and _recorder is not None:
            ev1 = TimingEvent() if _recorder.get("_native") else torch.cuda.Event(enable_timing=True)
            ev1.record(self.stream)
            _recorder.setdefault(self.what, []).append((self.ev0, ev1))  # type: ignore[union-attr]
        return False


def library_path() -> str:
    return _LIB_PATH


def load() -> ctypes.CDLL:
    """Open liboflow_hip.so once and declare the C signatures. Raises RuntimeError if it cannot."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(_LIB_PATH):
        raise RuntimeError(
            f"liboflow_hip.so not found at {_LIB_PATH}: build it with `make -C torch-optical-flow_amd/csrc` "
            "(or __graft_entry__.build()); the MI355X path has no CPU fallback"
        )
    lib = ctypes.CDLL(_LIB_PATH)
    P, I, F = ctypes.c_void_p, ctypes.c_int, ctypes.c_float
    IP = ctypes.POINTER(ctypes.c_int)
    PP = ctypes.POINTER(ctypes.c_void_p)
    lib.oflow_abi_version.restype = I
    lib.oflow_abi_version.argtypes = []
    lib.oflow_status_string.restype = ctypes.c_char_p
    lib.oflow_status_string.argtypes = [I]
    lib.oflow_corr_pyramid_dims.restype = I
    lib.oflow_corr_pyramid_dims.argtypes = [I, I, I, IP, IP]
    lib.oflow_corr_pyramid_f32.restype = I
    lib.oflow_corr_pyramid_f32.argtypes = [P, P, I, I, I, I, I, PP, P]
    lib.oflow_corr_lookup_f32.restype = I
    lib.oflow_corr_lookup_f32.argtypes = [PP, IP, IP, I, P, I, I, I, I, P, P]
    lib.oflow_corr_tiled_level_floats.restype = ctypes.c_longlong
    lib.oflow_corr_tiled_level_floats.argtypes = [I, I]
    lib.oflow_corr_pyramid_tiled_f32.restype = I
    lib.oflow_corr_pyramid_tiled_f32.argtypes = [P, P, I, I, I, I, I, PP, P]
    lib.oflow_corr_lookup_tiled_f32.restype = I
    lib.oflow_corr_lookup_tiled_f32.argtypes = [PP, IP, IP, I, P, I, I, I, I, P, P]
    lib.oflow_corr_untile_f32.restype = I
    lib.oflow_corr_untile_f32.argtypes = [P, P, ctypes.c_longlong, I, I, P]
    lib.oflow_grid_warp_f32.restype = I
    lib.oflow_grid_warp_f32.argtypes = [P, P, I, I, I, I, I, I, I, P, P]
    lib.oflow_grid_sample_f32.restype = I
    lib.oflow_grid_sample_f32.argtypes = [P, P, I, I, I, I, I, I, I, I, I, P, P]
    lib.oflow_corr_otf_prepare_f16.restype = I
    lib.oflow_corr_otf_prepare_f16.argtypes = [P, P, I, I, I, I, I, P, PP, P, P]
    L = ctypes.c_longlong
    lib.oflow_bias_act_f32.restype = I
    lib.oflow_bias_act_f32.argtypes = [P, L, P, P, L, P, L, I, I, I, I, F, P]
    lib.oflow_gru_reset_f32.restype = I
    lib.oflow_gru_reset_f32.argtypes = [P, L, P, P, L, P, L, I, I, I, P]
    lib.oflow_gru_blend_f32.restype = I
    lib.oflow_gru_blend_f32.argtypes = [P, L, P, P, L, P, P, L, I, I, I, P]
    lib.oflow_conv_s32.restype = I
    lib.oflow_conv_s32.argtypes = [P, L, I, P, I, P, P, I, I, I, I, I, I, I, I, I, F, P, L, P, L, P, L, L, I, P, P, I, P]
    lib.oflow_conv_s32_ex.restype = I
    lib.oflow_conv_s32_ex.argtypes = [P, L, I, P, I, P, P, I, I, I, I, I, I, I, I, I, F, P, L, P, L, P, L, L, I, P, P, I,
                                      P, I, P, P, L, I, I, P]
    lib.oflow_stem_patches_s32.restype = I
    lib.oflow_stem_patches_s32.argtypes = [P, I, I, I, I, P, I, P]
    lib.oflow_norm_stats_finalize.restype = I
    lib.oflow_norm_stats_finalize.argtypes = [P, I, I, I, I, ctypes.c_double, P, P, P]
    lib.oflow_norm_apply_s32.restype = I
    lib.oflow_norm_apply_s32.argtypes = [P, I, I, I, I, P, P, I, I, P, L, P, P, P, I, I, P, L, P]
    lib.oflow_pack_s32_f32.restype = I
    lib.oflow_pack_s32_f32.argtypes = [P, L, I, I, I, I, I, I, P, L, P, L, P, I, P]
    lib.oflow_flow_prep_s32.restype = I
    lib.oflow_flow_prep_s32.argtypes = [P, I, I, I, P, P, L, P, L, P]
    lib.oflow_corr_lookup_otf_f16.restype = I
    lib.oflow_corr_lookup_otf_f16.argtypes = [P, PP, IP, IP, I, P, I, I, I, I, I, P, P]
    lib.oflow_conv_s32_ex2.restype = I
    lib.oflow_conv_s32_ex2.argtypes = list(lib.oflow_conv_s32_ex.argtypes[:-1]) + [I, P, P, P]
    lib.oflow_conv_s32_ex3.restype = I
    lib.oflow_conv_s32_ex3.argtypes = list(lib.oflow_conv_s32_ex2.argtypes[:-1]) + [P, L, P]
    lib.oflow_conv_s32_ex4.restype = I
    lib.oflow_normalize_images_f32.restype = I
    lib.oflow_normalize_images_f32.argtypes = [P, P, L, P, P, P]
    lib.oflow_replicate_pad_f32.restype = I
    lib.oflow_replicate_pad_f32.argtypes = [P, P, I, L, I, I, I, I, I, I, P]
    lib.oflow_conv_s32_ex4.argtypes = list(lib.oflow_conv_s32_ex3.argtypes[:-1]) + [P, P]
    lib.oflow_conv_s32_ex5.restype = I
    lib.oflow_conv_s32_ex5.argtypes = list(lib.oflow_conv_s32_ex4.argtypes[:-1]) + [P, P, L, P]
    lib.oflow_corr_lookup_backward_f32.restype = I
    lib.oflow_corr_lookup_backward_f32.argtypes = [P, P, I, I, I, I, PP, IP, IP, I, P]
    lib.oflow_corr_pyramid_grad_combine_f32.restype = I
    lib.oflow_corr_pyramid_grad_combine_f32.argtypes = [PP, IP, IP, I, L, P]
    lib.oflow_corr_lookup_tiled_nhwc_f32.restype = I
    lib.oflow_corr_lookup_tiled_nhwc_f32.argtypes = [PP, IP, IP, I, P, I, I, I, I, P, I, P]
    lib.oflow_convex_upsample_f32.restype = I
    lib.oflow_flow_head2_s32.restype = I
    lib.oflow_flow_head2_s32.argtypes = [P, ctypes.c_longlong, I, P, P, I, I, I, P, P]
    lib.oflow_flow_head2_tiled_s32.restype = I
    lib.oflow_flow_head2_tiled_s32.argtypes = [P, ctypes.c_longlong, I, P, P, I, I, I, P, P]
    lib.oflow_corr_pyramid_tiled_s32.restype = I
    lib.oflow_corr_pyramid_tiled_s32.argtypes = [P, P, I, I, I, I, I, PP, P]
    lib.oflow_corr_lookup_convc1_s32.restype = I
    lib.oflow_corr_lookup_convc1_s32.argtypes = [PP, IP, IP, I, P, I, I, I, I, P, P, P, P, ctypes.c_longlong, P]
    lib.oflow_convex_upsample_f32.argtypes = [P, P, I, I, I, P, P]
    lib.oflow_flow_stats_f32.restype = I
    lib.oflow_flow_stats_f32.argtypes = [P, I, I, I, I, F, F, I, P, P]
    lib.oflow_flow2rgb_f32.restype = I
    lib.oflow_flow2rgb_f32.argtypes = [P, I, I, I, I, I, F, F, I, I, F, P, P, P]
    lib.oflow_flow_pack_f32.restype = I
    lib.oflow_flow_pack_f32.argtypes = [P, I, I, I, I, I, P, P]
    lib.oflow_set_range_flag.restype = I
    lib.oflow_set_range_flag.argtypes = [P]
    lib.oflow_range_flag_exchange.restype = I
    lib.oflow_range_flag_exchange.argtypes = [P, P, P]
    lib.oflow_timing_event_create.restype = I
    lib.oflow_timing_event_create.argtypes = [ctypes.POINTER(ctypes.c_void_p)]
    lib.oflow_timing_event_destroy.restype = I
    lib.oflow_timing_event_destroy.argtypes = [P]
    lib.oflow_timing_event_record.restype = I
    lib.oflow_timing_event_record.argtypes = [P, P, I]
    lib.oflow_timing_event_elapsed_ms.restype = I
    lib.oflow_timing_event_elapsed_ms.argtypes = [P, P, ctypes.POINTER(ctypes.c_float)]
    lib.oflow_flow_head_col2im_f32.restype = I
    lib.oflow_flow_head_col2im_f32.argtypes = [P, P, I, I, I, P, P]
    v = lib.oflow_abi_version()
    if v != ABI_VERSION:
        raise RuntimeError(f"liboflow_hip.so ABI version {v}, expected {ABI_VERSION}: rebuild the library")
    _ops.load()  # torch.ops.oflow.* (liboflow_torch.so over this library)
    _lib = lib
    return lib


def ops():
    """The ``torch.ops.oflow`` namespace (loads both libraries on first use)."""
    if _lib is None:
        load()
    return torch.ops.oflow


def _run(what: str, device: torch.device, op, *args):
    """``op(*args)``, bracketed by HIP events when the bench's recorder is on (kept out of traced graphs: with no
    recorder this is a plain call, so torch.compile sees only the op)."""
    if _recorder is None:
        return op(*args)
    with _Timed(what, device):
        return op(*args)


def _tensor(t, name: str, what: str) -> torch.Tensor:
    if not isinstance(t, torch.Tensor):
        raise TypeError(f"{what}: {name} must be a torch.Tensor")
    return t


def _no_grad_input(t: torch.Tensor, name: str, what: str) -> None:
    """Ops without an autograd formula (the inference layouts) refuse inputs that would need one."""
    if t.requires_grad and torch.is_grad_enabled():
        raise RuntimeError(
            f"{what}: {name} requires grad; this layout is inference-only (no backward): use CorrBlock's canonical "
            "pyramid (corr_pyramid / corr_lookup have autograd), or run under torch.no_grad()"
        )


def _check(status: int, what: str) -> None:
    if status == 0:
        return
    msg = load().oflow_status_string(status).decode()
    if status == E_TINY:
        raise ValueError(f"{what}: {msg}")
    raise RuntimeError(f"{what} failed ({status}): {msg}")


def _gpu_f32(t: torch.Tensor, name: str, what: str) -> torch.Tensor:
    if not isinstance(t, torch.Tensor):
        raise TypeError(f"{what}: {name} must be a torch.Tensor")
    if t.device.type != "cuda":
        raise RuntimeError(
            f"{what}: {name} is on {t.device}; this MI355X build runs only on ROCm GPU tensors (no CPU fallback)"
        )
    if t.requires_grad and torch.is_grad_enabled():
        # these raw entry points (tiled / NHWC / split-fp16 / on-the-fly layouts, the inference kernels) have no
        # autograd formula: fail loudly instead of returning a graph-less tensor. The differentiable path is the
        # canonical one (CorrBlock under autograd, optical_flow.warp / grid_sample: native backward kernels)
        raise RuntimeError(
            f"{what}: {name} requires grad; this entry point is an inference layout with no autograd formula: use "
            "CorrBlock / optical_flow.warp (native backward kernels), or run under torch.no_grad() / "
            "torch.inference_mode(), or detach the input"
        )
    if t.dtype != torch.float32:
        t = t.float()
    return t.contiguous()


def _stream(device: torch.device) -> ctypes.c_void_p:
    return ctypes.c_void_p(torch.cuda.current_stream(device).cuda_stream)


def pyramid_dims(h: int, w: int, num_levels: int):
    hs = (ctypes.c_int * MAX_LEVELS)()
    ws = (ctypes.c_int * MAX_LEVELS)()
    _check(load().oflow_corr_pyramid_dims(h, w, num_levels, hs, ws), "corr_pyramid_dims")
    return [(hs[i], ws[i]) for i in range(num_levels)]


def corr_pyramid(fmap1: torch.Tensor, fmap2: torch.Tensor, num_levels: int = 4) -> List[torch.Tensor]:
    """Level l of the all-pairs correlation pyramid as (B*H*W, 1, H_l, W_l) fp32 (``torch.ops.oflow.corr_pyramid``;
    differentiable in both feature maps)."""
    f1, f2 = _tensor(fmap1, "fmap1", "corr_pyramid"), _tensor(fmap2, "fmap2", "corr_pyramid")
    return list(_run("corr_pyramid", f1.device, ops().corr_pyramid, f1, f2, int(num_levels)))


class TiledPyramid:
    """Correlation pyramid in the tiled layout (include/oflow.h): level l is a (B*H*W, tiles_l*32) fp32 tensor,
    all levels views of one allocation; ``dims[l] = (H_l, W_l)``."""

    __slots__ = ("levels", "dims", "queries")

    def __init__(self, levels, dims, queries):
        self.levels, self.dims, self.queries = levels, dims, queries

    def batch_slice(self, b0: int, b1: int) -> "TiledPyramid":
        """Views of the pairs [b0, b1) (queries are pair-major, so each level's rows are one contiguous range)."""
        hw = self.dims[0][0] * self.dims[0][1]
        return TiledPyramid([t[b0 * hw : b1 * hw] for t in self.levels], self.dims, (b1 - b0) * hw)

    def untile(self, l: int) -> torch.Tensor:
        """Canonical (B*H*W, 1, H_l, W_l) copy of level l (the reference's corr_pyramid[l]), bit-exact."""
        hl, wl = self.dims[l]
        src = self.levels[l]
        out = torch.empty((self.queries, 1, hl, wl), device=src.device, dtype=torch.float32)
        if out.numel():
            with torch.cuda.device(src.device):
                _check(load().oflow_corr_untile_f32(src.data_ptr(), out.data_ptr(), self.queries, hl, wl, _stream(src.device)), "untile")
        return out


def corr_pyramid_tiled(fmap1: torch.Tensor, fmap2: torch.Tensor, num_levels: int = 4) -> TiledPyramid:
    """The all-pairs correlation pyramid (same values as ``corr_pyramid``) in the tiled lookup layout."""
    what = "corr_pyramid"
    f1, f2 = _tensor(fmap1, "fmap1", what), _tensor(fmap2, "fmap2", what)
    _no_grad_input(f1, "fmap1", what)
    _no_grad_input(f2, "fmap2", what)
    levels = list(_run(what, f1.device, ops().corr_pyramid_tiled, f1, f2, int(num_levels)))
    return TiledPyramid(levels, pyramid_dims(f1.shape[2], f1.shape[3], num_levels), int(levels[0].shape[0]))


def corr_pyramid_tiled_s32(f1: torch.Tensor, f2: torch.Tensor, num_levels: int = 4) -> TiledPyramid:
    """The tiled pyramid from S32 feature maps (B, H, W, C/32, 2, 32) (oflow_corr_pyramid_tiled_s32: split-fp16
    products, fp32 accumulation; the RAFT forward's pyramid)."""
    what = "corr_pyramid"
    for t in (f1, f2):
        if t.dtype != torch.float16 or t.dim() != 6 or tuple(t.shape[-2:]) != (2, 32) or not t.is_contiguous():
            raise RuntimeError(f"{what}: S32 feature maps must be contiguous fp16 (B, H, W, G, 2, 32)")
        if t.device.type != "cuda":
            raise RuntimeError(f"{what}: S32 feature maps must be on the GPU (no CPU fallback)")
    if f1.shape != f2.shape or f1.device != f2.device:
        raise RuntimeError(f"{what}: feature maps differ in shape or device")
    b, h, w, g = (int(v) for v in f1.shape[:4])
    dims = pyramid_dims(h, w, num_levels)
    lib = load()
    per_q = [int(lib.oflow_corr_tiled_level_floats(hl, wl)) for hl, wl in dims]
    q = b * h * w
    store = torch.empty((q * sum(per_q),), device=f1.device, dtype=torch.float32)
    levels, off = [], 0
    for n in per_q:
        levels.append(store[off * q : (off + n) * q].view(q, n))
        off += n
    ptrs = (ctypes.c_void_p * MAX_LEVELS)(*[t.data_ptr() for t in levels])
    if _flops is not None:  # the level-0 GEMM (pooling is the epilogue's)
        _count(3 * 2 * b * (h * w) ** 2 * g * 32, 2 * b * (h * w) ** 2 * g * 32)
    with torch.cuda.device(f1.device), _Timed(what, f1.device):
        _check(lib.oflow_corr_pyramid_tiled_s32(f1.data_ptr(), f2.data_ptr(), b, g * 32, h, w, int(num_levels), ptrs,
                                                _stream(f1.device)), what)
    return TiledPyramid(levels, dims, q)


def corr_lookup_tiled(pyr: TiledPyramid, coords: torch.Tensor, radius: int) -> torch.Tensor:
    """``corr_lookup`` on a ``TiledPyramid``: (B, L*(2r+1)^2, H, W) fp32 (``torch.ops.oflow.corr_lookup_tiled``)."""
    co = _tensor(coords, "coords", "corr_lookup")
    _no_grad_input(co, "coords", "corr_lookup")
    return _run("corr_lookup", co.device, ops().corr_lookup_tiled, pyr.levels, co, int(radius))


def corr_lookup(levels: Sequence[torch.Tensor], coords: torch.Tensor, radius: int) -> torch.Tensor:
    """(B, L*(2r+1)^2, H, W) fp32 windowed lookup of ``levels`` at ``coords`` (B, 2, H, W)
    (``torch.ops.oflow.corr_lookup``; differentiable in the levels, coords get no gradient as in the reference)."""
    co = _tensor(coords, "coords", "corr_lookup")
    return _run("corr_lookup", co.device, ops().corr_lookup, list(levels), co.detach(), int(radius))


def _modes(mode: str, padding_mode: str, what: str):
    if mode not in INTERP:
        raise ValueError(f"{what}: nn.functional.grid_sample(): expected mode to be 'bilinear', 'nearest' or 'bicubic', but got: '{mode}'")
    if padding_mode not in PADDING:
        raise ValueError(
            f"{what}: nn.functional.grid_sample(): expected padding_mode to be 'zeros', 'border', or 'reflection', but got: '{padding_mode}'"
        )
    return INTERP[mode], PADDING[padding_mode]


def grid_warp(frame: torch.Tensor, flow: torch.Tensor, mode: str, padding_mode: str, align_corners: bool) -> torch.Tensor:
    """grid_sample(frame, linspace-grid + flow) with the grid never materialised (``torch.ops.oflow.grid_warp``;
    differentiable in frame and flow)."""
    what = "warp"
    m, p = _modes(mode, padding_mode, what)
    fr, fl = _tensor(frame, "frame", what), _tensor(flow, "flow", what)
    return _run("grid_warp", fr.device, ops().grid_warp, fr, fl, m, p, bool(align_corners))


def convex_upsample(flow: torch.Tensor, mask: torch.Tensor) -> torch.Tensor:
    """RAFT.upsample_flow (methods/raft/model/raft.py:73-85): flow (B, 2, H, W), mask (B, 576, H, W) ->
    (B, 2, 8H, 8W), one fused kernel (softmax over 9 neighbours x unfold(8 * flow) x sum x permute)."""
    what = "upsample_flow"
    fl = _gpu_f32(flow, "flow", what)
    mk = _gpu_f32(mask, "mask", what)
    if fl.dim() != 4 or fl.shape[1] != 2 or mk.dim() != 4 or mk.shape[1] != 576 or mk.shape[0] != fl.shape[0] or mk.shape[2:] != fl.shape[2:]:
        raise RuntimeError(f"{what}: flow {tuple(flow.shape)} must be (B, 2, H, W) and mask {tuple(mask.shape)} (B, 576, H, W)")
    if fl.device != mk.device:
        raise RuntimeError(f"{what}: flow and mask are on different devices")
    b, _, h, w = fl.shape
    out = torch.empty((b, 2, 8 * h, 8 * w), device=fl.device, dtype=torch.float32)
    if out.numel() == 0:
        return out
    with torch.cuda.device(fl.device), _Timed("upsample_flow", fl.device):
        _check(load().oflow_convex_upsample_f32(fl.data_ptr(), mk.data_ptr(), b, h, w, out.data_ptr(), _stream(fl.device)), what)
    return out


FLOW2RGB_METHODS = {"baker": 0, "hsv": 1, "meister": 2}
FLOW_STATS_CHUNKS = 128  # include/oflow.h OFLOW_FLOW_STATS_CHUNKS


def _flow_b2hw(flow: torch.Tensor, what: str) -> torch.Tensor:
    fl = _gpu_f32(flow, "flow", what)
    if fl.dim() != 4 or fl.shape[1] != 2:
        raise RuntimeError(f"{what}: flow {tuple(flow.shape)} must be (B, 2, H, W)")
    return fl


def flow2rgb(flow: torch.Tensor, method: str, clip, denom, invert_y: bool) -> torch.Tensor:
    """optical_flow.flow2rgb (optical_flow/visualization/flow2rgb.py:19-73) on (B, 2, H, W) fp32: clip (None or a
    (lo, hi) pair), y inversion, division by ``denom`` (the fp32 value of max_norm + 1e-5; None = per image
    max |flow| + 1e-5) and the baker / hsv / meister colour map, in two launches (flow_stats, flow2rgb) ->
    (B, 3, H, W) fp32."""
    what = "flow2rgb"
    if method not in FLOW2RGB_METHODS:
        raise ValueError(f"Unknown method: '{method}'.")
    fl = _flow_b2hw(flow, what)
    b, _, h, w = fl.shape
    out = torch.empty((b, 3, h, w), device=fl.device, dtype=torch.float32)
    if out.numel() == 0:
        return out
    do_clip = clip is not None
    lo, hi = (float(clip[0]), float(clip[1])) if do_clip else (0.0, 0.0)
    have_denom = denom is not None
    denom = float(denom) if have_denom else 0.0
    need_stats = (not have_denom) or method == "meister"
    lib = load()
    with torch.cuda.device(fl.device), _Timed("flow2rgb", fl.device):
        stream = _stream(fl.device)
        parts = None
        if need_stats:
            parts = torch.empty((b, FLOW_STATS_CHUNKS, 2), device=fl.device, dtype=torch.float32)
            _check(lib.oflow_flow_stats_f32(fl.data_ptr(), b, h, w, int(do_clip), lo, hi, int(bool(invert_y)),
                                            parts.data_ptr(), stream), what)
        _check(lib.oflow_flow2rgb_f32(fl.data_ptr(), b, h, w, FLOW2RGB_METHODS[method], int(do_clip), lo, hi,
                                      int(bool(invert_y)), int(have_denom), denom,
                                      parts.data_ptr() if parts is not None else None, out.data_ptr(), stream), what)
    return out


def flow_pack(flow: torch.Tensor, channels: int, flip_rows: bool) -> torch.Tensor:
    """Planar (B, 2, H, W) flow -> the file payload (B, H, W, channels) fp32 on the device: channels 2 = Middlebury
    .flo rows (optical_flow/io/middlebury.py:64-71), 3 = PFM rows (zero third channel, bottom-up when flip_rows;
    optical_flow/io/pfm.py:95-98)."""
    what = "flow_pack"
    fl = _flow_b2hw(flow, what)
    b, _, h, w = fl.shape
    out = torch.empty((b, h, w, channels), device=fl.device, dtype=torch.float32)
    if out.numel() == 0:
        return out
    with torch.cuda.device(fl.device), _Timed("flow_pack", fl.device):
        _check(load().oflow_flow_pack_f32(fl.data_ptr(), b, h, w, int(channels), int(bool(flip_rows)),
                                          out.data_ptr(), _stream(fl.device)), what)
    return out


def grid_sample(inp: torch.Tensor, grid: torch.Tensor, mode: str, padding_mode: str, align_corners: bool) -> torch.Tensor:
    """F.grid_sample for 4-D input (B, C, H, W) and grid (B, Ho, Wo, 2) (``torch.ops.oflow.grid_sample``)."""
    what = "grid_sample"
    m, p = _modes(mode, padding_mode, what)
    x, g = _tensor(inp, "input", what), _tensor(grid, "grid", what)
    return _run("grid_sample", x.device, ops().grid_sample, x, g, m, p, bool(align_corners))


def otf_prepare(fmap1: torch.Tensor, fmap2: torch.Tensor, num_levels: int = 4):
    """fmap1/sqrt(C) and the floor-pooled fmap2 pyramid as NHWC fp16 tensors (on-the-fly correlation inputs).
    Returns (f1h (B, H, W, C), [f2h_l (B, H_l, W_l, C)])."""
    what = "corr_otf_prepare"
    f1, f2 = _tensor(fmap1, "fmap1", what), _tensor(fmap2, "fmap2", what)
    _no_grad_input(f1, "fmap1", what)
    _no_grad_input(f2, "fmap2", what)
    f1h, f2h = _run(what, f1.device, ops().corr_otf_prepare, f1, f2, int(num_levels))
    return f1h, list(f2h)


def corr_lookup_otf(f1h: torch.Tensor, f2h: Sequence[torch.Tensor], coords: torch.Tensor, radius: int) -> torch.Tensor:
    """(B, L*(2r+1)^2, H, W) fp32 lookup computed from the fp16 feature pyramid, no correlation volume."""
    co = _tensor(coords, "coords", "corr_lookup_otf")
    _no_grad_input(co, "coords", "corr_lookup_otf")
    return _run("corr_lookup_otf", co.device, ops().corr_lookup_otf, f1h, list(f2h), co, int(radius))


ACT = {"none": 0, "relu": 1, "sigmoid": 2, "tanh": 3}

# Range guard of the split-fp16 operands (always on): every kernel that writes or stages S32 values sets a sticky
# device flag when a value's hi half would overflow fp16 (|x| >= 65520 or inf; include/oflow.h oflow_set_range_flag).
# The RAFT forward reads it once (RAFT.range_guard) and raises; no per-convolution reduction or sync.
_range_flags = {}


def range_flag(device: torch.device) -> torch.Tensor:
    """The device's range flag (one int32, registered with the library on first use for that device)."""
    device = torch.device(device)
    idx = device.index if device.index is not None else torch.cuda.current_device()
    flag = _range_flags.get(idx)
    if flag is None:
        flag = torch.zeros(1, dtype=torch.int32, device=torch.device("cuda", idx))
        with torch.cuda.device(idx):
            torch.cuda.synchronize(idx)  # the zero fill is complete before any kernel may set it
            _check(load().oflow_set_range_flag(ctypes.c_void_p(flag.data_ptr())), "set_range_flag")
        _range_flags[idx] = flag
    return flag


class RangeSnapshot:
    """One forward's split-fp16 range status: the device's range flag exchanged with 0 on the forward's stream right
    after its kernels (oflow_range_flag_exchange), copied into pinned host memory; ``event`` is recorded after the copy.
    One per forward."""

    __slots__ = ("dev_word", "host", "event", "device")

    def __init__(self, device: torch.device) -> None:
        self.device = device
        self.dev_word = torch.empty(1, dtype=torch.int32, device=device)
        self.host = torch.empty(1, dtype=torch.int32, pin_memory=True)
        self.event = torch.cuda.Event()

    def take(self) -> "RangeSnapshot":
        """Enqueue the exchange + copy on the current stream of the device."""
        flag = range_flag(self.device)
        stream = torch.cuda.current_stream(self.device)
        with torch.cuda.device(self.device):
            _check(load().oflow_range_flag_exchange(ctypes.c_void_p(flag.data_ptr()),
                                                    ctypes.c_void_p(self.dev_word.data_ptr()),
                                                    ctypes.c_void_p(stream.cuda_stream)), "range_flag_exchange")
            self.host.copy_(self.dev_word, non_blocking=True)
            self.event.record(stream)
        return self

    def done(self) -> bool:
        return self.event.query()

    def overflowed(self) -> bool:
        """Wait for the snapshot and return whether the forward (or one running concurrently) overflowed."""
        self.event.synchronize()
        return bool(int(self.host[0]))


RANGE_ERROR = ("a split-fp16 operand exceeded the fp16 range (|x| >= 65520) -- an activation outside the range these "
               "kernels represent exactly; the output is not valid (OFLOW_CHECK=1 names the convolution)")


def range_flag_raise_if_set(device: torch.device, what: str = "RAFT forward", all_streams: bool = False) -> None:
    """Read the device's range flag (one D2H copy of 4 bytes: a sync of the current stream, or of the whole device with
    ``all_streams``: forwards in flight on other streams) and raise if a split-fp16 operand overflowed since the last
    check; the flag is cleared before raising."""
    device = torch.device(device)
    if all_streams:
        torch.cuda.synchronize(device)
    if RangeSnapshot(device).take().overflowed():  # read and clear in one exchange (nothing set meanwhile is lost)
        raise RuntimeError(f"{what}: {RANGE_ERROR}")


# OFLOW_CHECK=1: before every split-fp16 convolution, a device-side max-abs reduction over its input (the values that
# become fp16 hi + lo operands) raises if any |x| > 65504, where the hi half would overflow to inf. Debug mode: one
# reduction and one host sync per convolution. Off by default (the checked RAFT activations stay below ~1e3).
CHECK_RANGE = os.environ.get("OFLOW_CHECK", "0") not in ("", "0")
F16_MAX = 65504.0
# conv_s32 passes the fragment-major weights (ConvWeights.frag) to the 128-channel multi-tap convolutions: their B
# operand goes to registers straight from HBM / L2 instead of through LDS (csrc/conv_s32.hip, BREG). Bit-identical.
CONV_BREG = True
# ... and (off: measured not faster; the tests exercise both) to the 64-channel 3x3 blocks
# (2 x 2 waves, each two row tiles x one 32-channel tile) and to the 32-channel 3x3 blocks (4 x 1 waves)
CONV_BREG64 = False
CONV_BREG32 = False


def _range_check(x, what: str) -> None:
    if isinstance(x, S32Slice):  # already split: an overflowed hi half is inf
        v = x.t[:, :, :, x.g0 : x.g0 + x.ng, 0]
    elif isinstance(x, NhwcNormIn):  # the kernel stages relu(raw * scale + shift)
        b, h, w = x.bhw
        c = x.raw.shape[1]
        v = torch.relu(x.raw.view(b, h * w, c) * x.scale.view(b, 1, c) + x.shift.view(b, 1, c))
    else:
        v = x.raw
    m = float(v.abs().amax().float()) if v.numel() else 0.0
    if not m <= F16_MAX:
        raise RuntimeError(
            f"{what}: input max |x| = {m:g} is outside the fp16 range (65504) of the split-fp16 operands (OFLOW_CHECK)"
        )


def _chan_view(t: torch.Tensor, what: str):
    """(B, C, H, W) fp32 CUDA tensor whose (C, H, W) part is contiguous -> (ptr, batch stride, C, P)."""
    if t.device.type != "cuda" or t.dtype != torch.float32 or t.dim() != 4:
        raise RuntimeError(f"{what}: expected a 4-D fp32 ROCm tensor, got {t.dtype} {tuple(t.shape)} on {t.device}")
    b, c, h, w = t.shape
    if t.stride(3) != 1 or t.stride(2) != w or t.stride(1) != h * w:
        raise RuntimeError(f"{what}: the (C, H, W) part must be contiguous")
    return t.data_ptr(), t.stride(0), c, h * w


def bias_act_(x: torch.Tensor, bias, act: str = "relu", scale: float = 1.0, out=None, out2=None) -> torch.Tensor:
    """out = act(x + bias[c]) * scale (in place when out is None); optionally also into out2."""
    px, sx, c, p = _chan_view(x, "bias_act")
    y = x if out is None else out
    py, sy, cy, py_ = _chan_view(y, "bias_act out")
    p2, s2 = (0, 0)
    if out2 is not None:
        p2, s2, c2, _ = _chan_view(out2, "bias_act out2")
        if c2 != c:
            raise RuntimeError("bias_act: out2 channel count differs")
    if cy != c or py_ != p or y.shape[0] != x.shape[0]:
        raise RuntimeError("bias_act: output shape differs from input")
    if bias is not None and (bias.numel() != c or bias.dtype != torch.float32 or not bias.is_contiguous()):
        raise RuntimeError("bias_act: bias must be a contiguous fp32 vector of C elements")
    with torch.cuda.device(x.device):
        _check(
            load().oflow_bias_act_f32(
                px, sx, bias.data_ptr() if bias is not None else None, py, sy, p2 or None, s2, x.shape[0], c, p,
                ACT[act], float(scale), _stream(x.device)
            ),
            "bias_act",
        )
    return y


def gru_reset(zr: torch.Tensor, br: torch.Tensor, h: torch.Tensor, rh: torch.Tensor) -> None:
    """rh = sigmoid(zr[:, CH:] + br) * h  (zr = [z | r] pre-bias, CH = h channels)."""
    pz, sz, c2, p = _chan_view(zr, "gru_reset zr")
    ph, sh, ch, p1 = _chan_view(h, "gru_reset h")
    pr, sr, cr, p2 = _chan_view(rh, "gru_reset rh")
    if c2 != 2 * ch or cr != ch or p1 != p or p2 != p or br.numel() != ch:
        raise RuntimeError("gru_reset: inconsistent shapes")
    with torch.cuda.device(h.device):
        _check(load().oflow_gru_reset_f32(pz, sz, br.data_ptr(), ph, sh, pr, sr, h.shape[0], ch, p, _stream(h.device)), "gru_reset")


def gru_blend_(zr: torch.Tensor, bz: torch.Tensor, q: torch.Tensor, bq: torch.Tensor, h: torch.Tensor) -> None:
    """h <- (1 - z) * h + z * tanh(q + bq), z = sigmoid(zr[:, :CH] + bz), in place."""
    pz, sz, c2, p = _chan_view(zr, "gru_blend zr")
    pq, sq, cq, p1 = _chan_view(q, "gru_blend q")
    ph, sh, ch, p2 = _chan_view(h, "gru_blend h")
    if c2 != 2 * ch or cq != ch or p1 != p or p2 != p or bz.numel() != ch or bq.numel() != ch:
        raise RuntimeError("gru_blend: inconsistent shapes")
    with torch.cuda.device(h.device):
        _check(
            load().oflow_gru_blend_f32(pz, sz, bz.data_ptr(), pq, sq, bq.data_ptr(), ph, sh, h.shape[0], ch, p, _stream(h.device)),
            "gru_blend",
        )


# ---- split-fp16 ("S32") update-block path (include/oflow.h; csrc/conv_s32.hip, s32_io.hip) -------------------
# An S32 activation tensor is fp16 (B, H, W, G, 2, 32): per pixel and 32-channel group one 128-B line holding
# hi = fp16(v) then lo = fp16(v - hi). A channel slice is ``S32Slice(tensor, g0, ng)``.


class S32Slice:
    """Groups [g0, g0 + ng) of an S32 tensor (a channel slice of a concatenated buffer)."""

    __slots__ = ("t", "g0", "ng")

    def __init__(self, t: torch.Tensor, g0: int = 0, ng: int = -1):
        if t.dtype != torch.float16 or t.dim() != 6 or tuple(t.shape[-2:]) != (2, 32) or not t.is_contiguous():
            raise RuntimeError(f"S32 tensor must be contiguous fp16 (B, H, W, G, 2, 32), got {t.dtype} {tuple(t.shape)}")
        self.t, self.g0 = t, int(g0)
        self.ng = int(t.shape[3]) - self.g0 if ng < 0 else int(ng)
        if self.g0 < 0 or self.g0 + self.ng > t.shape[3]:
            raise RuntimeError("S32Slice: group range outside the tensor")

    @property
    def ptr(self) -> int:
        return self.t.data_ptr() + self.g0 * 128

    @property
    def ps(self) -> int:
        return int(self.t.shape[3]) * 128

    def channel_ptr(self, c: int) -> int:
        """Byte address of the hi half of channel c of the slice."""
        return self.ptr + (c // 32) * 128 + (c % 32) * 2

    @property
    def bhw(self):
        return tuple(int(v) for v in self.t.shape[:3])

    @property
    def device(self):
        return self.t.device


class F32In:
    """Convolution input given as a dense fp32 NHWC tensor [B*H*W, C] (C % 4 == 0; the channels past C up to the next
    multiple of 32 stage as zeros), split into hi + lo while the kernel stages it (oflow_conv_s32_ex2, OFLOW_IN_F32;
    1x1 convs): the RAFT forward's lookup rows (corr_lookup_tiled_nhwc, C = L*(2r+1)^2 = 324)."""

    __slots__ = ("raw", "bhw")
    in_format = 2

    def __init__(self, raw: torch.Tensor, b: int, h: int, w: int):
        if raw.dtype != torch.float32 or not raw.is_contiguous() or raw.shape[0] != b * h * w or raw.shape[1] % 4:
            raise RuntimeError("F32In: raw must be contiguous fp32 [B*H*W, C], C % 4 == 0")
        self.raw, self.bhw = raw, (int(b), int(h), int(w))

    @property
    def ptr(self) -> int:
        return self.raw.data_ptr()

    @property
    def ps(self) -> int:
        return int(self.raw.shape[1]) * 4

    @property
    def ng(self) -> int:
        return (int(self.raw.shape[1]) + 31) // 32

    @property
    def device(self):
        return self.raw.device


class ImgIn:
    """The encoders' stem input given as the fp32 NCHW image (B, 3, 2H, 2W) itself (OFLOW_IN_IMG7S2): the 7x7/2 pad-3
    conv's patch operand is built per output tile from the staged input window, so no patch matrix is written. For
    ConvWeights packed with ``patches=True`` (5 groups); the output is (B, H, W)."""

    __slots__ = ("raw", "bhw")
    in_format = 3

    def __init__(self, img: torch.Tensor):
        if img.dtype != torch.float32 or img.dim() != 4 or img.shape[1] != 3 or not img.is_contiguous():
            raise RuntimeError("ImgIn: the image must be contiguous fp32 (B, 3, H, W)")
        b, _, hh, ww = img.shape
        if hh % 2 or ww % 2:
            raise RuntimeError("ImgIn: H and W must be even")
        self.raw, self.bhw = img, (int(b), int(hh) // 2, int(ww) // 2)

    @property
    def ptr(self) -> int:
        return self.raw.data_ptr()

    @property
    def ps(self) -> int:
        return 0

    @property
    def ng(self) -> int:
        return 5

    @property
    def device(self):
        return self.raw.device


class FlowIn:
    """convf1's input given as coords1 (B, 2, H, W) fp32 itself (OFLOW_IN_FLOW7): flow = coords1 - the pixel grid
    and its 7x7 pad-3 patch operand are built per output tile from a staged window, so no patch matrix is written or
    read. For ConvWeights packed with ``patches=True`` (4 groups); bit-identical to the conv of flow_prep's matrix."""

    __slots__ = ("raw", "bhw")
    in_format = 4

    def __init__(self, coords: torch.Tensor):
        if coords.dtype != torch.float32 or coords.dim() != 4 or coords.shape[1] != 2 or not coords.is_contiguous():
            raise RuntimeError("FlowIn: coords must be contiguous fp32 (B, 2, H, W)")
        b, _, hh, ww = coords.shape
        self.raw, self.bhw = coords, (int(b), int(hh), int(ww))

    @property
    def ptr(self) -> int:
        return self.raw.data_ptr()

    @property
    def ps(self) -> int:
        return 0

    @property
    def ng(self) -> int:
        return 4

    @property
    def device(self):
        return self.raw.device


class NhwcNormIn:
    """Convolution input given as the previous convolution's raw fp32 NHWC output [B*H*W, C] plus its instance-norm
    affine (scale, shift: [B, C]); the kernel stages relu(raw * scale + shift) (oflow_conv_s32_ex2), so the normalised
    activation is never written to HBM."""

    __slots__ = ("raw", "bhw", "scale", "shift")
    in_format = 1

    def __init__(self, raw: torch.Tensor, b: int, h: int, w: int, scale: torch.Tensor, shift: torch.Tensor):
        c = raw.shape[1]
        if raw.dtype != torch.float32 or not raw.is_contiguous() or raw.shape[0] != b * h * w or c % 32:
            raise RuntimeError("NhwcNormIn: raw must be contiguous fp32 [B*H*W, C], C % 32 == 0")
        for t in (scale, shift):
            if t.dtype != torch.float32 or not t.is_contiguous() or t.numel() != b * c:
                raise RuntimeError("NhwcNormIn: scale / shift must be contiguous fp32 [B, C]")
        self.raw, self.bhw, self.scale, self.shift = raw, (int(b), int(h), int(w)), scale, shift

    @property
    def ptr(self) -> int:
        return self.raw.data_ptr()

    @property
    def ps(self) -> int:
        return int(self.raw.shape[1]) * 4

    @property
    def ng(self) -> int:
        return int(self.raw.shape[1]) // 32

    @property
    def device(self):
        return self.raw.device


def s32_empty(b: int, h: int, w: int, groups: int, device, zero: bool = False) -> torch.Tensor:
    f = torch.zeros if zero else torch.empty
    return f((b, h, w, groups, 2, 32), device=device, dtype=torch.float16)


def s32_from_f32(x: torch.Tensor, groups: int = -1) -> torch.Tensor:
    """(B, C, H, W) fp32 -> S32 tensor (torch ops; test / reference helper, not on the hot path)."""
    b, c, h, w = x.shape
    g = (c + 31) // 32 if groups < 0 else groups
    v = torch.zeros((b, h, w, g * 32), device=x.device, dtype=torch.float32)
    v[..., :c] = x.permute(0, 2, 3, 1)
    hi = v.half()
    lo = (v - hi.float()).half()
    return torch.stack([hi.view(b, h, w, g, 32), lo.view(b, h, w, g, 32)], dim=4).contiguous()


def s32_to_f32(t: torch.Tensor, channels: int = -1) -> torch.Tensor:
    """S32 tensor -> (B, C, H, W) fp32 = hi + lo."""
    b, h, w, g = t.shape[:4]
    v = (t[:, :, :, :, 0].float() + t[:, :, :, :, 1].float()).reshape(b, h, w, g * 32)
    c = g * 32 if channels < 0 else channels
    return v[..., :c].permute(0, 3, 1, 2).contiguous()


class ConvWeights:
    """A conv layer's weights packed for oflow_conv_s32: [in_groups][taps][n_pad][hi | lo] fp16 (per-output-channel
    power-of-two scaled so that max |w| = 2^14 keeps the lo halves normal), the inverse scales and the bias."""

    __slots__ = ("pack", "wscale", "bias", "n", "n_pad", "kh", "kw", "kg", "layout", "cin", "_frag")

    def __init__(self, weight: torch.Tensor, bias, n_pad: int, patches: bool = False):
        w = weight.detach().float()
        if patches:  # kh x kw conv as a 1x1 over its patch matrix (flow_prep, stem_patches): channel k = t*C + c
            n, c, kh, kw = w.shape
            w = w.permute(0, 2, 3, 1).reshape(n, kh * kw * c, 1, 1)
        n, c, kh, kw = w.shape
        if n_pad < n:
            raise RuntimeError("ConvWeights: n_pad < out channels")
        amax = w.abs().amax(dim=(1, 2, 3))
        e = torch.where(amax > 0, torch.ceil(torch.log2(amax)), torch.zeros_like(amax)).clamp(-100, 100)
        scale = torch.exp2(14.0 - e)
        ws = w * scale.view(-1, 1, 1, 1)
        kg = (c + 31) // 32
        t = kh * kw
        full = torch.zeros((n_pad, kg * 32, t), device=w.device, dtype=torch.float32)
        full[:n, :c] = ws.reshape(n, c, t)
        full = full.view(n_pad, kg, 32, t).permute(1, 3, 0, 2).contiguous()  # [kg][t][n_pad][32]
        hi = full.half()
        lo = (full - hi.float()).half()
        self.pack = torch.stack([hi, lo], dim=3).contiguous()  # [kg][t][n_pad][2][32]
        inv = torch.ones(n_pad, device=w.device, dtype=torch.float32)
        inv[:n] = 1.0 / scale
        self.wscale = inv
        self.bias = None if bias is None else bias.detach().float().contiguous()
        self.n, self.n_pad, self.kh, self.kw, self.kg = n, n_pad, kh, kw, kg
        self.cin = c  # real input channels (flop accounting)
        self.layout = "conv"  # "convc1_frag": convc1_level_weights (the fused lookup + convc1's fragment-major order)
        self._frag = None
        if t > 1 and n_pad % 32 == 0:  # built with the pack, never lazily inside a captured / timed forward
            self.frag()

    def frag(self) -> torch.Tensor:
        """The pack reordered fragment-major for oflow_conv_s32_ex4's register-direct weights (include/oflow.h):
        [kg][t][n_pad][hi, lo][k 32] -> [kg][t][n / 32][sub-step][hi, lo][k half][n % 32][8], built once."""
        if self._frag is None:
            if self.layout != "conv" or self.n_pad % 32:
                raise RuntimeError("ConvWeights.frag: needs a conv-layout pack with n_pad a multiple of 32")
            kg, t = self.pack.shape[:2]
            f = self.pack.reshape(kg, t, self.n_pad // 32, 32, 2, 2, 2, 8)  # kg, t, ntile, r, hi/lo, sub, hh, 8
            self._frag = f.permute(0, 1, 2, 5, 4, 6, 3, 7).contiguous()
        return self._frag


def convc1_level_weights(conv: torch.nn.Conv2d, num_levels: int, radius: int) -> "ConvWeights":
    """convc1 (1x1, L*(2r+1)^2 -> 256) packed for oflow_corr_lookup_convc1_s32: input channel l*(2r+1)^2 + k (the
    lookup's channel order, corr.py:71-77) moved to l*G*32 + k, G = ceil((2r+1)^2 / 32), zeros between levels."""
    kk = (2 * radius + 1) ** 2
    g = (kk + 31) // 32
    w = conv.weight.detach().float()
    if tuple(w.shape[1:]) != (num_levels * kk, 1, 1):
        raise RuntimeError(f"convc1_level_weights: expected a 1x1 conv over {num_levels * kk} channels, got {tuple(w.shape)}")
    wp = w.new_zeros((w.shape[0], num_levels * g * 32, 1, 1))
    for l in range(num_levels):
        wp[:, l * g * 32 : l * g * 32 + kk] = w[:, l * kk : (l + 1) * kk]
    cw = ConvWeights(wp, conv.bias, w.shape[0])
    # fragment-major (include/oflow.h): [group][n 256][hi, lo][k 32] -> [group][wave][ntile][sub][hi, lo][hh][r][8]
    lg = cw.pack.shape[0]
    frag = cw.pack.reshape(lg, 4, 2, 32, 2, 2, 2, 8)  # group, wave, ntile, r, hi/lo, sub, hh, 8
    cw.pack = frag.permute(0, 1, 2, 5, 4, 6, 3, 7).contiguous()
    cw.layout = "convc1_frag"
    cw.cin = num_levels * kk
    return cw


def corr_lookup_convc1(pyr: "TiledPyramid", coords: torch.Tensor, radius: int, cw: "ConvWeights", y: "S32Slice") -> None:
    """relu(convc1(lookup(coords))) straight into the S32 slice ``y`` (256 channels), the lookup fused into the
    convolution (oflow_corr_lookup_convc1_s32): the RAFT forward's `F.relu(self.convc1(corr_fn(coords1)))`
    (raft.py:128, update.py:120-121). ``cw``: ``convc1_level_weights``."""
    what = "corr_lookup_convc1"
    co = _gpu_f32(coords, "coords", what)
    b, two, h, w = co.shape
    if two != 2 or b * h * w != pyr.queries:
        raise RuntimeError(f"{what}: coords (B, 2, H, W) must cover the pyramid's {pyr.queries} queries")
    kk = (2 * radius + 1) ** 2
    if (cw.layout != "convc1_frag" or cw.n != 256 or cw.n_pad != 256 or cw.kh * cw.kw != 1
            or cw.kg != len(pyr.levels) * ((kk + 31) // 32)):
        raise RuntimeError(f"{what}: weights must be convc1_level_weights of this pyramid / radius")
    if y.ng != 8 or y.bhw != (b, h, w) or y.device != co.device:
        raise RuntimeError(f"{what}: destination must be an 8-group S32 slice of shape ({b}, {h}, {w})")
    n = len(pyr.levels)
    ptrs = (ctypes.c_void_p * MAX_LEVELS)(*[t.data_ptr() for t in pyr.levels])
    hs = (ctypes.c_int * MAX_LEVELS)(*[d[0] for d in pyr.dims])
    ws = (ctypes.c_int * MAX_LEVELS)(*[d[1] for d in pyr.dims])
    if _flops is not None:
        _count(3 * 2 * b * h * w * 256 * cw.kg * 32, 2 * b * h * w * 256 * cw.cin)
    with torch.cuda.device(co.device), _Timed(what, co.device):
        _check(
            load().oflow_corr_lookup_convc1_s32(
                ptrs, hs, ws, n, co.data_ptr(), b, h, w, int(radius), cw.pack.data_ptr(), cw.wscale.data_ptr(),
                cw.bias.data_ptr() if cw.bias is not None else None, y.ptr, y.ps, _stream(co.device),
            ),
            what,
        )


def conv_tiles(h: int, w: int) -> int:
    """Output tiles (4 rows x 32 columns) per image of oflow_conv_s32: the instance-norm partials' tile count."""
    return ((h + 3) // 4) * ((w + 31) // 32)


class KSplit:
    """Split-K scratch for oflow_conv_s32_ex5 (include/oflow.h): an fp32 partial slab of ``tiles`` (4 x 32-pixel tile,
    128-channel block) units and its [ticket, published] counters, zeroed here once. Calls sharing one KSplit must be
    stream-ordered (one per update lane)."""

    def __init__(self, b: int, h: int, w: int, device, block_n: int = 128, blocks: int = 1) -> None:
        self.tiles = b * conv_tiles(h, w) * blocks  # (blocks: channel blocks of block_n per tile)
        self.block_n = block_n
        self.slab = torch.empty(self.tiles * 128 * block_n, device=device, dtype=torch.float32)
        self.ctr = torch.zeros(2 * self.tiles, device=device, dtype=torch.int32)


def conv_s32(x: S32Slice, cw: ConvWeights, block_n: int, act: str = "none", out_scale: float = 1.0, y0=None, y1=None,
             f32=None, f32_accumulate: bool = False, epilogue: int = 0, gru_h=None, gru_z=None, nhwc=None, stats=None,
             res=None, res_act: str = "none", s2d: bool = False, addend=None, ksplit: "KSplit" = None) -> None:
    """Split-fp16 convolution (oflow_conv_s32_ex5). x: input S32Slice with cw.kg groups, or NhwcNormIn (3x3 only). y0/y1: S32Slice destinations
    (s2d: space-to-depth layout, half the spatial size). f32: (B, N', H, W) fp32 NCHW destination. nhwc: [P, N]
    fp32 destination. stats: instance-norm partials [B, conv_tiles(H, W), n_pad, 3]. res: S32Slice residual added
    after the activation, then res_act. epilogue 1/2: GRU gates / candidate with gru_h, gru_z ([P, CH] fp32);
    addend: fp32 [P, >= N] (row stride a multiple of 4, 16-B aligned) added before the gate activations (the GRU's
    hoisted context term). ksplit: split-K scratch (KSplit) -- the register-direct kernels then run each tile as two
    workgroups over half the input groups each (one more fp32 addition per output); other kernels ignore it."""
    what = "conv_s32"
    if CHECK_RANGE:
        _range_check(x, f"{what} {cw.kh}x{cw.kw}")
    if x.ng != cw.kg:
        raise RuntimeError(f"{what}: input has {x.ng} groups, weights expect {cw.kg}")
    b, h, w = x.bhw
    nin = isinstance(x, NhwcNormIn)
    in_format = getattr(x, "in_format", 0)
    hw_out = (h // 2, w // 2) if s2d else (h, w)
    for d in (y0, y1):
        if d is not None and (tuple(d.t.shape[:3]) != (b, *hw_out) or d.t.device != x.device):
            raise RuntimeError(f"{what}: destination shape/device mismatch")
    if res is not None and (tuple(res.t.shape[:3]) != (b, h, w) or res.ng * 32 < cw.n):
        raise RuntimeError(f"{what}: residual shape mismatch")
    fp, fbs, fcs = 0, 0, 0
    if f32 is not None:
        if f32.dtype != torch.float32 or f32.dim() != 4 or tuple(f32.shape[2:]) != (h, w) or f32.shape[0] != b:
            raise RuntimeError(f"{what}: fp32 destination must be (B, C, H, W) fp32")
        if f32.stride(3) != 1 or f32.stride(2) != w or f32.shape[1] < cw.n and epilogue == 0:
            raise RuntimeError(f"{what}: fp32 destination planes must be contiguous with >= N channels")
        fp, fbs, fcs = f32.data_ptr(), f32.stride(0), f32.stride(1)
    if nhwc is not None and (nhwc.dtype != torch.float32 or not nhwc.is_contiguous() or nhwc.numel() != b * h * w * cw.n):
        raise RuntimeError(f"{what}: nhwc destination must be contiguous fp32 [P, {cw.n}]")
    if stats is not None and (stats.dtype != torch.float32 or stats.numel() < b * conv_tiles(h, w) * cw.n_pad * 3):
        raise RuntimeError(f"{what}: stats partials buffer too small")
    gh = gz = 0
    gch = 0
    if epilogue:
        gch = cw.n // 2 if epilogue == 1 else cw.n
        for tt in (gru_h, gru_z):
            if tt is None or tt.dtype != torch.float32 or not tt.is_contiguous() or tt.numel() != b * h * w * gch:
                raise RuntimeError(f"{what}: GRU state tensors must be contiguous fp32 [P, {gch}]")
        gh, gz = gru_h.data_ptr(), gru_z.data_ptr()
    ap, aps = 0, 0
    if addend is not None:
        if (not epilogue or addend.dtype != torch.float32 or addend.dim() != 2 or addend.stride(1) != 1
                or addend.shape[0] != b * h * w or addend.shape[1] < cw.n or addend.stride(0) % 4
                or addend.data_ptr() % 16 or addend.device != x.device):
            raise RuntimeError(f"{what}: addend must be a GRU-epilogue fp32 [P, >= {cw.n}] view with 16-B aligned rows")
        ap, aps = addend.data_ptr(), addend.stride(0)
    dev = x.device
    # register-direct weights for the 128- (and, CONV_BREG64, 64-) channel blocks of multi-tap convs on S32 input (the
    # kernel ignores wf elsewhere)
    wf = (cw.frag().data_ptr() if CONV_BREG and (int(block_n) == 128 or (CONV_BREG64 and int(block_n) == 64)
                                                 or (CONV_BREG32 and int(block_n) == 32))
          and cw.kh * cw.kw > 1 and not nin
          and in_format == 0 and cw.layout == "conv" else None)
    if _flops is not None:
        taps, p_out = cw.kh * cw.kw, b * h * w  # (s2d only changes where the epilogue writes)
        n_exec = -(-cw.n_pad // int(block_n)) * int(block_n)
        _count(3 * 2 * p_out * n_exec * cw.kg * 32 * taps, 2 * p_out * cw.n * cw.cin * taps)
    ks_slab = ks_ctr = None
    ks_tiles = 0
    if ksplit is not None and wf is not None:
        if ksplit.slab.device != dev or ksplit.block_n < int(block_n):
            raise RuntimeError(f"{what}: split-K scratch on another device or for narrower channel blocks")
        ks_slab, ks_ctr = ksplit.slab.data_ptr(), ksplit.ctr.data_ptr()
        ks_tiles = ksplit.tiles * (ksplit.block_n // int(block_n))
    with torch.cuda.device(dev), _Timed(f"conv{cw.kh}x{cw.kw}", dev):
        _check(
            load().oflow_conv_s32_ex5(
                x.ptr, x.ps, cw.kg, cw.pack.data_ptr(), cw.n_pad, cw.wscale.data_ptr(),
                cw.bias.data_ptr() if cw.bias is not None else None, cw.n, b, h, w, cw.kh, cw.kw, int(block_n),
                int(epilogue), ACT[act], float(out_scale), y0.ptr if y0 is not None else None, y0.ps if y0 is not None else 0,
                y1.ptr if y1 is not None else None, y1.ps if y1 is not None else 0, fp or None, fbs, fcs,
                int(bool(f32_accumulate)), gh or None, gz or None, gch,
                nhwc.data_ptr() if nhwc is not None else None, cw.n,
                stats.data_ptr() if stats is not None else None,
                res.ptr if res is not None else None, res.ps if res is not None else 0, ACT[res_act], int(bool(s2d)),
                in_format, x.scale.data_ptr() if nin else None, x.shift.data_ptr() if nin else None,
                ap or None, aps, wf, ks_slab, ks_ctr, ks_tiles, _stream(dev),
            ),
            what,
        )


def flow_head2(x: "S32Slice", weight: torch.Tensor, bias: torch.Tensor, coords: torch.Tensor) -> None:
    """coords += conv3x3(x, weight, bias) for the flow head's 2-channel output conv as fp32 FMAs (oflow_flow_head2_s32;
    update.py:36, raft.py:133), the small-grid form. x: S32Slice of C <= 256 channels; weight (2, C, 3, 3) fp32
    contiguous; coords (B, 2, H, W) fp32 contiguous."""
    what = "flow_head2"
    b, h, w = x.bhw
    if weight.dtype != torch.float32 or not weight.is_contiguous() or tuple(weight.shape) != (2, x.ng * 32, 3, 3):
        raise RuntimeError(f"{what}: weight must be contiguous fp32 (2, {x.ng * 32}, 3, 3)")
    if bias is None or bias.dtype != torch.float32 or tuple(bias.shape) != (2,):
        raise RuntimeError(f"{what}: bias must be fp32 (2,)")
    if coords.dtype != torch.float32 or not coords.is_contiguous() or tuple(coords.shape) != (b, 2, h, w):
        raise RuntimeError(f"{what}: coords must be contiguous fp32 ({b}, 2, {h}, {w})")
    if _flops is not None:
        fl = 2 * b * h * w * 2 * x.ng * 32 * 9
        _count(0, fl, fl)
    with torch.cuda.device(coords.device), _Timed("conv3x3", coords.device):
        _check(load().oflow_flow_head2_s32(x.ptr, x.ps, x.ng, weight.data_ptr(), bias.data_ptr(), b, h, w,
                                           coords.data_ptr(), _stream(coords.device)), what)


def flow_head2_tiled_weights(weight: torch.Tensor) -> torch.Tensor:
    """(2, C, 3, 3) fp32 -> the [group][4-channel chunk][tap][output][4] copy oflow_flow_head2_tiled_s32 reads."""
    o, c = weight.shape[:2]
    if o != 2 or c % 32 or tuple(weight.shape[2:]) != (3, 3):
        raise RuntimeError("flow_head2_tiled_weights: weight must be (2, C, 3, 3) with C a multiple of 32")
    w = weight.detach().float().reshape(2, c // 32, 8, 4, 3, 3)  # o, g, c4, e, ky, kx
    return w.permute(1, 2, 4, 5, 0, 3).contiguous()  # g, c4, ky, kx, o, e


def flow_head2_tiled(x: "S32Slice", wr: torch.Tensor, bias: torch.Tensor, coords: torch.Tensor) -> None:
    """coords += conv3x3(x, weight, bias) for the flow head's 2-channel output conv as fp32 FMAs on an LDS-staged halo
    (oflow_flow_head2_tiled_s32; update.py:36, raft.py:133), the large-grid form. wr: flow_head2_tiled_weights(weight)."""
    what = "flow_head2_tiled"
    b, h, w = x.bhw
    if wr.dtype != torch.float32 or not wr.is_contiguous() or wr.numel() != 2 * x.ng * 32 * 9 or wr.data_ptr() % 16:
        raise RuntimeError(f"{what}: wr must be flow_head2_tiled_weights of a (2, {x.ng * 32}, 3, 3) weight")
    if bias is None or bias.dtype != torch.float32 or tuple(bias.shape) != (2,):
        raise RuntimeError(f"{what}: bias must be fp32 (2,)")
    if coords.dtype != torch.float32 or not coords.is_contiguous() or tuple(coords.shape) != (b, 2, h, w):
        raise RuntimeError(f"{what}: coords must be contiguous fp32 ({b}, 2, {h}, {w})")
    if _flops is not None:
        fl = 2 * b * h * w * 2 * x.ng * 32 * 9
        _count(0, fl, fl)
    with torch.cuda.device(coords.device), _Timed("conv3x3", coords.device):
        _check(load().oflow_flow_head2_tiled_s32(x.ptr, x.ps, x.ng, wr.data_ptr(), bias.data_ptr(), b, h, w,
                                                 coords.data_ptr(), _stream(coords.device)), what)


def flow_head_col2im(y: torch.Tensor, bias: torch.Tensor, coords: torch.Tensor) -> None:
    """coords += bias + the 3x3 gather of the per-tap products y (B, 18, H, W) (oflow_flow_head_col2im_f32): the flow
    head's output conv as 1x1 conv C -> 18 + col2im (update.py:36, raft.py:133)."""
    what = "flow_head_col2im"
    b, _, h, w = coords.shape
    if coords.dtype != torch.float32 or not coords.is_contiguous() or coords.shape[1] != 2 or coords.device.type != "cuda":
        raise RuntimeError(f"{what}: coords must be contiguous fp32 (B, 2, H, W) on the GPU")
    if y.dtype != torch.float32 or not y.is_contiguous() or tuple(y.shape) != (b, 18, h, w) or y.device != coords.device:
        raise RuntimeError(f"{what}: y must be contiguous fp32 ({b}, 18, {h}, {w})")
    if bias is None or bias.dtype != torch.float32 or tuple(bias.shape) != (2,) or bias.device != coords.device:
        raise RuntimeError(f"{what}: bias must be fp32 (2,) on the coords' device")
    with torch.cuda.device(coords.device), _Timed("flow_head_col2im", coords.device):
        _check(load().oflow_flow_head_col2im_f32(y.data_ptr(), bias.data_ptr(), b, h, w, coords.data_ptr(),
                                                 _stream(coords.device)), what)


def stem_patches(img: torch.Tensor, out: torch.Tensor) -> torch.Tensor:
    """7x7 / stride 2 / pad 3 patch matrix of a (B, C, H, W) fp32 image as S32 (channel t*C + c)."""
    x = _gpu_f32(img, "image", "stem_patches")
    b, c, h, w = x.shape
    if out.dtype != torch.float16 or tuple(out.shape[:3]) != (b, (h + 1) // 2, (w + 1) // 2):
        raise RuntimeError("stem_patches: output must be S32 (B, ceil(H/2), ceil(W/2), G, 2, 32)")
    with torch.cuda.device(x.device), _Timed("stem_patches", x.device):
        _check(load().oflow_stem_patches_s32(x.data_ptr(), b, c, h, w, out.data_ptr(), int(out.shape[3]), _stream(x.device)), "stem_patches")
    return out


def norm_stats(partials: torch.Tensor, b: int, tiles: int, n_pad: int, c: int, eps: float):
    """Per-(image, channel) instance-norm affine (alpha = 1/sqrt(var + eps), beta = -mean * alpha) from partials."""
    alpha = torch.empty((b, c), device=partials.device, dtype=torch.float32)
    beta = torch.empty_like(alpha)
    with torch.cuda.device(partials.device):
        _check(
            load().oflow_norm_stats_finalize(partials.data_ptr(), b, tiles, n_pad, c, float(eps), alpha.data_ptr(), beta.data_ptr(), _stream(partials.device)),
            "norm_stats",
        )
    return alpha, beta


def norm_apply(x: torch.Tensor, shape, alpha, beta, act: str, y: S32Slice, res=None, res_raw=None, res_act: str = "none",
               s2d: bool = False, res_raw_relu: bool = False) -> None:
    """y = act(x*alpha + beta) (+ residual, res_act) as S32. x: [P, C] fp32 (NHWC). res: S32Slice (identity shortcut);
    res_raw: (x2 [P, C], alpha2, beta2) normalised shortcut (relu'd first when res_raw_relu)."""
    b, c, h, w = shape
    mode, rp, rps = 0, None, 0
    x2 = a2 = b2 = None
    if res is not None:
        mode, rp, rps = 1, res.ptr, res.ps
    elif res_raw is not None:
        mode = 3 if res_raw_relu else 2
        x2, a2, b2 = (t.data_ptr() for t in res_raw)
    with torch.cuda.device(x.device), _Timed("norm_apply", x.device):
        _check(
            load().oflow_norm_apply_s32(
                x.data_ptr(), c, b, h, w, alpha.data_ptr(), beta.data_ptr(), ACT[act], mode, rp, rps, x2, a2, b2,
                ACT[res_act], int(bool(s2d)), y.ptr, y.ps, _stream(x.device),
            ),
            "norm_apply",
        )


def pack_s32(x: torch.Tensor, act: str, y0: S32Slice, y1=None, nhwc=None, dst_channel: int = 0) -> None:
    """(B, C, H, W) fp32 (a channel slice of a contiguous tensor is fine) -> act -> channels dst_channel + c of the S32
    slices (dst_channel % 8 == 0; the last 8-channel chunk is zero-filled past C), optionally also [P, C] fp32."""
    what = "pack_s32"
    if x.device.type != "cuda" or x.dtype != torch.float32 or x.dim() != 4:
        raise RuntimeError(f"{what}: expected a 4-D fp32 ROCm tensor")
    b, c, h, w = x.shape
    if x.stride(3) != 1 or x.stride(2) != w or x.stride(1) != h * w:
        raise RuntimeError(f"{what}: the (C, H, W) part must be contiguous")
    need = dst_channel + ((c + 7) // 8) * 8
    if dst_channel % 8 or y0.ng * 32 < need or (y1 is not None and y1.ng * 32 < need):
        raise RuntimeError(f"{what}: destination slice too narrow or dst_channel not a multiple of 8")
    if nhwc is not None and (nhwc.dtype != torch.float32 or not nhwc.is_contiguous() or nhwc.numel() != b * h * w * c):
        raise RuntimeError(f"{what}: nhwc copy must be contiguous fp32 [P, C]")
    with torch.cuda.device(x.device):
        _check(
            load().oflow_pack_s32_f32(
                x.data_ptr(), x.stride(0), c, b, h, w, ACT[act], int(dst_channel), y0.ptr, y0.ps,
                y1.ptr if y1 is not None else None, y1.ps if y1 is not None else 0,
                nhwc.data_ptr() if nhwc is not None else None, c, _stream(x.device),
            ),
            what,
        )


def normalize_images(image0: torch.Tensor, image1: torch.Tensor):
    """RAFT.forward's `2 * (image / 255.0) - 1.0` for both frames in one kernel (oflow_normalize_images_f32: the
    reference's fp32 operations with a correctly rounded division, bit-identical to the reference on the CPU -- ATen on
    the GPU multiplies by fl(1/255) instead). Same-shape fp32 GPU tensors; returns new contiguous ones."""
    what = "normalize_images"
    x0 = _gpu_f32(image0, "image0", what).contiguous()
    x1 = _gpu_f32(image1, "image1", what).contiguous()
    if x0.shape != x1.shape or x0.device != x1.device:
        raise RuntimeError(f"{what}: the frames must have the same shape and device")
    y0, y1 = torch.empty_like(x0), torch.empty_like(x1)
    n = x0.numel()
    with torch.cuda.device(x0.device):
        _check(load().oflow_normalize_images_f32(x0.data_ptr(), x1.data_ptr(), n, y0.data_ptr(), y1.data_ptr(),
                                                 _stream(x0.device)), what)
    return y0, y1


def replicate_pad(inputs, pad):
    """F.pad(x, pad, mode="replicate") (pad = [left, right, top, bottom]) of 1..4 same-shape fp32 GPU tensors of >= 2
    dims in one launch (oflow_replicate_pad_f32; a copy, bit-exact). Returns new contiguous tensors."""
    what = "replicate_pad"
    xs = [_gpu_f32(x, "input", what).contiguous() for x in inputs]  # (strided inputs: copied first)
    if not 1 <= len(xs) <= 4 or any(x.shape != xs[0].shape or x.device != xs[0].device for x in xs) or xs[0].dim() < 2:
        raise RuntimeError(f"{what}: 1..4 tensors of one shape (>= 2 dims) on one device")
    left, right, top, bottom = (int(v) for v in pad)
    *lead, h, w = xs[0].shape
    outs = [torch.empty((*lead, h + top + bottom, w + left + right), device=xs[0].device, dtype=torch.float32) for _ in xs]
    planes = xs[0].numel() // (h * w)
    src = (ctypes.c_void_p * len(xs))(*[x.data_ptr() for x in xs])
    dst = (ctypes.c_void_p * len(xs))(*[o.data_ptr() for o in outs])
    with torch.cuda.device(xs[0].device):
        _check(load().oflow_replicate_pad_f32(src, dst, len(xs), planes, h, w, top, bottom, left, right,
                                              _stream(xs[0].device)), what)
    return outs


def flow_prep(coords: torch.Tensor, patches: Optional[torch.Tensor], flow0=None, flow1=None) -> None:
    """coords1 (B, 2, H, W) -> convf1 patch matrix (S32, 4 groups; None: not written, convf1 reading coords1 through
    ``FlowIn``) and the flow channels of the GRU inputs. flow0/flow1: (S32Slice, channel) pairs naming where the x flow
    channel lives (y follows it)."""
    co = _gpu_f32(coords, "coords", "flow_prep")
    b, _, h, w = co.shape
    if patches is None and flow0 is None:
        raise RuntimeError("flow_prep: nothing to write")
    if patches is not None and (tuple(patches.shape) != (b, h, w, 4, 2, 32) or patches.dtype != torch.float16):
        raise RuntimeError("flow_prep: patches must be S32 (B, H, W, 4, 2, 32)")
    f0 = (flow0[0].channel_ptr(flow0[1]), flow0[0].ps) if flow0 is not None else (None, 0)
    f1 = (flow1[0].channel_ptr(flow1[1]), flow1[0].ps) if flow1 is not None else (None, 0)
    with torch.cuda.device(co.device), _Timed("flow_prep", co.device):
        _check(load().oflow_flow_prep_s32(co.data_ptr(), b, h, w, patches.data_ptr() if patches is not None else None,
                                          f0[0], f0[1], f1[0], f1[1], _stream(co.device)), "flow_prep")


def corr_lookup_backward(grad_out: torch.Tensor, coords: torch.Tensor, radius: int, level0_hw, num_levels: int):
    """The lookup's input gradient: the transpose of corr_lookup for the same coords (which get no gradient, as in
    the reference), as new canonical levels (B*H*W, 1, H_l, W_l) fp32 for a level-0 size ``level0_hw``."""
    h0, w0 = level0_hw
    return list(ops().corr_lookup_backward(grad_out, coords, int(radius), int(h0), int(w0), int(num_levels)))


def corr_pyramid_backward(level_grads, fmap1: torch.Tensor, fmap2: torch.Tensor):
    """(grad_fmap1, grad_fmap2) from the pyramid level gradients: the floor-pool transpose (native kernel) and two
    batched GEMMs."""
    return tuple(ops().corr_pyramid_backward(list(level_grads), fmap1, fmap2))


def corr_lookup_tiled_nhwc(pyr: TiledPyramid, coords: torch.Tensor, radius: int, out: torch.Tensor) -> torch.Tensor:
    """``corr_lookup_tiled`` as fp32 NHWC rows into ``out`` [B*H*W, row] (row >= L*(2r+1)^2; 16-B aligned), in the
    reference's channel order (row q = ``corr[b, :, y, x]``); channels past L*(2r+1)^2 are left untouched. With
    row = L*(2r+1)^2 this is exactly ``CorrBlock.__call__(coords).permute(0, 2, 3, 1)``: convc1's input (F32In)."""
    co = _tensor(coords, "coords", "corr_lookup")
    _no_grad_input(co, "coords", "corr_lookup")
    _run("corr_lookup", co.device, ops().corr_lookup_tiled_nhwc, pyr.levels, co, int(radius), out)
    return out