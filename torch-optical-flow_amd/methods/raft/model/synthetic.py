"""Deterministic synthetic inputs for RAFT inference: hash weights and integer texture frames.

No checkpoint or dataset is reachable offline (`pretrained/download.sh:3-6` needs the
network), so parity fixtures, smoke runs and the bench all use weights and frames that any machine can
regenerate bit-for-bit from integer arithmetic alone:

* weights: splitmix64 over ``(param_index << 32) + element_index`` (state_dict order), top 24 bits -> u in
  [0, 1), scaled per parameter class. Encoder convs get the variance of the
  reference's ``kaiming_normal_(mode="fan_out")`` init (`extractor.py:190-192`), update-block convs and all
  biases torch's default ``1/sqrt(fan_in)`` bound, norms 1/0, BN running stats 0/1.
* frames: an integer-valued RGB texture on a half-pixel lattice (two octaves of integer-bilinear hash noise),
  frame 1 = frame 0 displaced by a sub-pixel shift, so the true flow is known and the values are the 0..255
  integers a decoded 8-bit image holds (`predict.py:30-31`).
"""
from __future__ import annotations

from typing import Dict, Iterable, Tuple

import numpy as np
import torch

_M64 = np.uint64(0xFFFFFFFFFFFFFFFF)


def splitmix64(x: np.ndarray) -> np.ndarray:
    """splitmix64 finaliser on a uint64 array (wrapping arithmetic)."""
    with np.errstate(over="ignore"):
        z = (x.astype(np.uint64) + np.uint64(0x9E3779B97F4A7C15)) & _M64
        z = ((z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)) & _M64
        z = ((z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)) & _M64
        return z ^ (z >> np.uint64(31))


def hash_uniform(stream: int, numel: int, offset: int = 0) -> np.ndarray:
    """``numel`` float64 values in [0, 1) from stream ``stream`` (24-bit resolution, exact in fp32)."""
    idx = (np.uint64(stream) << np.uint64(32)) + np.arange(offset, offset + numel, dtype=np.uint64)
    bits = splitmix64(idx) >> np.uint64(40)
    return bits.astype(np.float64) / float(1 << 24)


def hash_normal(stream: int, shape: Iterable[int], std: float = 1.0) -> np.ndarray:
    """Approximately normal float32 samples (Irwin-Hall, 4 uniforms), mean 0, std ``std``.

    Only exact float64 sums of 24-bit uniforms and one correctly rounded multiply are used, so the values
    are bit-identical on every machine (no libm transcendental whose last ulp may differ by CPU).
    """
    shape = tuple(int(s) for s in shape)
    n = int(np.prod(shape)) if shape else 1
    s = np.zeros(n, dtype=np.float64)
    for k in range(4):
        s += hash_uniform(4 * stream + k + 1, n)
    return ((s - 2.0) * (std * np.sqrt(3.0))).astype(np.float32).reshape(shape)


def _fans(shape: Tuple[int, ...]) -> Tuple[int, int]:
    receptive = int(np.prod(shape[2:])) if len(shape) > 2 else 1
    return shape[1] * receptive, shape[0] * receptive


def synthetic_state_dict(template: Dict[str, torch.Tensor]) -> Dict[str, torch.Tensor]:
    """Hash-initialised copy of a RAFT ``state_dict`` (same keys/shapes/dtypes as ``template``).

    Classification follows SURVEY.md Appendix A.2: a 4-D ``.weight`` is a conv weight; a ``.bias`` whose
    ``.weight`` is 4-D is a conv bias; 1-D ``.weight``/``.bias`` belong to a norm (``downsample.1`` is a BN,
    so classify by rank, not by name).
    """
    out: Dict[str, torch.Tensor] = {}
    for pidx, (key, ref) in enumerate(template.items()):
        shape = tuple(ref.shape)
        if key.endswith("num_batches_tracked"):
            out[key] = ref.clone()
            continue
        if key.endswith("running_mean"):
            out[key] = torch.zeros_like(ref)
            continue
        if key.endswith("running_var"):
            out[key] = torch.ones_like(ref)
            continue
        base = key.rsplit(".", 1)[0]
        wkey = base + ".weight"
        wshape = tuple(template[wkey].shape) if wkey in template else shape
        if len(wshape) == 4:  # conv weight or conv bias
            fan_in, fan_out = _fans(wshape)
            u = hash_uniform(pidx, int(np.prod(shape)))
            if key.endswith(".weight") and (key.startswith("fnet.") or key.startswith("cnet.")):
                bound = np.sqrt(6.0 / fan_out)
            else:
                bound = 1.0 / np.sqrt(fan_in)
            vals = ((2.0 * u - 1.0) * bound).astype(np.float32).reshape(shape)
            out[key] = torch.from_numpy(vals).to(ref.dtype)
        elif key.endswith(".weight"):
            out[key] = torch.ones_like(ref)
        else:
            out[key] = torch.zeros_like(ref)
    return out


def _octave(u: np.ndarray, v: np.ndarray, spacing: int, stream: int) -> np.ndarray:
    """Integer-bilinear interpolation of hash lattice values in 0..255 (exact integer arithmetic)."""
    iu, fu = np.divmod(u, spacing)
    iv, fv = np.divmod(v, spacing)

    def lattice(a: np.ndarray, b: np.ndarray) -> np.ndarray:
        key = ((a.astype(np.int64) & 0xFFFF) << 16) | (b.astype(np.int64) & 0xFFFF)
        h = splitmix64((np.uint64(stream) << np.uint64(32)) + key.astype(np.uint64))
        return (h >> np.uint64(56)).astype(np.int64)  # 0..255

    p00, p01 = lattice(iu, iv), lattice(iu + 1, iv)
    p10, p11 = lattice(iu, iv + 1), lattice(iu + 1, iv + 1)
    s = spacing
    acc = p00 * (s - fu) * (s - fv) + p01 * fu * (s - fv) + p10 * (s - fu) * fv + p11 * fu * fv
    return acc // (s * s)


def texture(u: np.ndarray, v: np.ndarray, channel: int, seed: int) -> np.ndarray:
    """Integer texture in 0..255 at half-pixel lattice coordinates (u, v) = (2x, 2y)."""
    base = 1000 + 16 * seed + 4 * channel
    coarse = _octave(u, v, 48, base)
    fine = _octave(u, v, 12, base + 1)
    return (3 * coarse + fine) // 4


def synthetic_pair(
    batch: int,
    height: int,
    width: int,
    shift: Tuple[float, float] = (3.0, -1.5),
    seed: int = 0,
) -> Tuple[torch.Tensor, torch.Tensor]:
    """Frames (B, 3, H, W) float32, integer-valued 0..255; frame1(x) = frame0(x - shift).

    ``shift`` must be a multiple of 0.5 px (the texture lives on a half-pixel lattice). Pair ``b`` uses
    texture seed ``seed + b`` so batch elements differ.
    """
    du, dv = 2.0 * shift[0], 2.0 * shift[1]
    if du != int(du) or dv != int(dv):
        raise ValueError("shift must be a multiple of 0.5 px")
    du, dv = int(du), int(dv)
    ys, xs = np.meshgrid(np.arange(height, dtype=np.int64), np.arange(width, dtype=np.int64), indexing="ij")
    u0, v0 = 2 * xs, 2 * ys
    img0 = np.empty((batch, 3, height, width), dtype=np.float32)
    img1 = np.empty_like(img0)
    for b in range(batch):
        for c in range(3):
            img0[b, c] = texture(u0, v0, c, seed + b)
            img1[b, c] = texture(u0 - du, v0 - dv, c, seed + b)
    return torch.from_numpy(img0), torch.from_numpy(img1)


def synthetic_fmaps(batch: int, dim: int, height: int, width: int, stream: int = 7, std: float = 1.45):
    """Feature maps ~ N(0, std^2) (the measured fnet output std) as float32 tensors."""
    f1 = hash_normal(stream, (batch, dim, height, width), std)
    f2 = hash_normal(stream + 100, (batch, dim, height, width), std)
    return torch.from_numpy(f1), torch.from_numpy(f2)
