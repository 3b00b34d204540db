"""Oracle: flow visualisation and flow-file payloads on the CPU. TEST INFRASTRUCTURE ONLY.

Restates optical_flow/visualization/flow2rgb.py:19-73 with its colour maps (visualization/methods/baker.py:32-146,
hsv.py:8-36, meister.py:30-55, utils.py:19-61) and the writers' payloads (io/middlebury.py:43-71,
io/pfm.py:79-104) as plain per-element fp32 arithmetic on NumPy, one array op per reference op so the roundings
are the reference's. Pinned by tests/golden/io_small.npz (made by the reference itself, gen_goldens.py io).
"""
from __future__ import annotations

import numpy as np

EPS = np.float32(1e-5)
PI = np.float32(np.pi)
TWO_PI = np.float32(2 * np.pi)


def baker_wheel() -> np.ndarray:
    """(55, 3) colour wheel, `baker.py:81-146`: segments RY 15, YG 6, GC 4, CB 11, BM 13, MR 6; ramps floor(255 i / n)."""
    # (length, channel held at 255, ramped channel, ramp direction)
    segs = [(15, 0, 1, +1), (6, 1, 0, -1), (4, 1, 2, +1), (11, 2, 1, -1), (13, 2, 0, +1), (6, 0, 2, -1)]
    wheel = np.zeros((55, 3), np.float32)
    row = 0
    for n, full, ramp_ch, sign in segs:
        ramp = np.floor(255.0 * np.arange(n) / n)
        wheel[row:row + n, full] = 255
        wheel[row:row + n, ramp_ch] = ramp if sign > 0 else 255 - ramp
        row += n
    return wheel


def _hsv_to_rgb(h, s, v):
    """`utils.py:19-61` per element: sector hi = floor(6h) mod 6, f = (6h mod 6) - hi."""
    f32 = np.float32
    h6 = (h * f32(6)).astype(np.float32)
    hi = np.mod(np.floor(h6), f32(6))
    f = (np.mod(h6, f32(6)) - hi).astype(np.float32)
    p = v * (f32(1) - s)
    q = v * (f32(1) - f * s)
    t = v * (f32(1) - (f32(1) - f) * s)
    table = [(v, t, p), (q, v, p), (p, v, t), (p, q, v), (t, p, v), (v, p, q)]
    hi = hi.astype(np.int64)
    out = np.zeros((3,) + h.shape, np.float32)
    for k, (r, g, b) in enumerate(table):
        m = hi == k
        for c, src in enumerate((r, g, b)):
            out[c][m] = src[m]
    return out


def flow2rgb(flow: np.ndarray, method: str = "baker", clip=None, max_norm=None, invert_y: bool = False) -> np.ndarray:
    """(B, 2, H, W) or (2, H, W) fp32 -> (B, 3, H, W) / (3, H, W) in [0, 1] (`flow2rgb.py:19-73`)."""
    f32 = np.float32
    flow = np.array(flow, dtype=np.float32, copy=True)
    squeeze = flow.ndim == 3
    if squeeze:
        flow = flow[None]
    if clip is not None:
        lo, hi = (-clip, clip) if not isinstance(clip, tuple) else clip
        flow = np.minimum(np.maximum(flow, f32(lo)), f32(hi))
    if invert_y:
        flow[:, 1] *= f32(-1)
    if max_norm is None:
        norm = np.sqrt(flow[:, 0] * flow[:, 0] + flow[:, 1] * flow[:, 1])
        d = (norm.reshape(flow.shape[0], -1).max(axis=1) + EPS).astype(np.float32)[:, None, None, None]
    else:
        d = f32(max_norm + 1e-5)
    flow = (flow / d).astype(np.float32)
    u, v = flow[:, 0], flow[:, 1]
    if method == "baker":  # `baker.py:54-74`
        wheel = baker_wheel()
        a = np.arctan2(-v, -u) / PI
        fk = (a + f32(1)) / f32(2) * f32(54)
        k0 = np.floor(fk).astype(np.int64)
        k1 = np.where(k0 + 1 == 55, 0, k0 + 1)
        fr = (fk - k0.astype(np.float32)).astype(np.float32)
        rad = np.sqrt(u * u + v * v)
        out = np.empty((3,) + u.shape, np.float32)
        for c in range(3):
            col0 = wheel[k0, c] / f32(255)
            col1 = wheel[k1, c] / f32(255)
            col = (f32(1) - fr) * col0 + fr * col1
            col = np.where(rad <= 1, f32(1) - rad * (f32(1) - col), col * f32(0.75))
            out[c] = np.floor(f32(255) * col) / f32(255)
    elif method == "hsv":  # `hsv.py:21-35`
        dx, dy = u, -v
        angle = np.arctan2(dy, dx)
        angle = np.where(angle < 0, angle + TWO_PI, angle).astype(np.float32)
        sc = np.sqrt(dx * dx + dy * dy)
        s = np.clip(sc, f32(0), f32(1))
        out = _hsv_to_rgb((angle / TWO_PI).astype(np.float32), s, np.ones_like(s))
    elif method == "meister":  # `meister.py:43-54`
        mag = np.sqrt(u * u + v * v)
        angle = np.arctan2(v, u)
        max_flow = flow.reshape(flow.shape[0], -1).max(axis=1)[:, None, None]
        h = np.mod(angle / TWO_PI + f32(1), f32(1)).astype(np.float32)
        s = np.clip(mag * f32(8) / max_flow, f32(0), f32(1)).astype(np.float32)
        val = np.clip(f32(8) - s, f32(0), f32(1)).astype(np.float32)
        out = _hsv_to_rgb(h, s, val)
    else:
        raise ValueError(f"Unknown method: '{method}'.")
    out = np.moveaxis(out, 0, 1).astype(np.float32)
    return out[0] if squeeze else out


def flo_bytes(flow: np.ndarray) -> bytes:
    """Middlebury .flo file of a (2, H, W) flow: magic 202021.25, width, height, (H, W, 2) rows (`middlebury.py:60-71`)."""
    _, h, w = flow.shape
    body = np.ascontiguousarray(np.asarray(flow, np.float32).transpose(1, 2, 0))
    return np.float32(202021.25).tobytes() + np.array([w, h], np.int32).tobytes() + body.tobytes()


def pfm_bytes(flow: np.ndarray) -> bytes:
    """PFM file of a (2, H, W) flow: header, then (H, W, 3) rows with a zero third channel, bottom row first
    (`pfm.py:95-104`; little-endian host -> scale -1)."""
    _, h, w = flow.shape
    body = np.asarray(flow, np.float32).transpose(1, 2, 0)[::-1]
    body = np.concatenate((body, np.zeros_like(body[..., :1])), -1)
    return f"PF\n{w:d} {h:d}\n{-1:f}\n".encode() + np.ascontiguousarray(body).tobytes()
