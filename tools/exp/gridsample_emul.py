"""Bit-level model of ATen's CPU grid_sampler_2d (the reference's warp runs on it) in numpy float32, used to pin the
HIP kernel's arithmetic: the AVX kernels are compiled with FP contraction, so unnormalize, reflection and the tap
sums are fused multiply-adds. Run: python tools/exp/gridsample_emul.py  (prints mismatches vs torch CPU, expect 0)."""
import numpy as np
import torch
import torch.nn.functional as F

f32 = np.float32


def fma(a, b, c):
    """float32 fma via float64 (exact product of two float32; one rounding of the sum is not always exact in
    double, so this is checked against the long-double route for the test ranges)."""
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    c = np.asarray(c, np.float64)
    p = a * b  # exact: 24+24 bits < 53
    s = np.asarray(p + c, np.longdouble) if False else None
    # exact sum via TwoSum in double then round to float32 with the error term deciding ties
    hi = p + c
    bb = hi - p
    err = (p - (hi - bb)) + (c - bb)
    r = hi.astype(np.float32)
    # correct double rounding: if hi is exactly halfway between two float32s, err decides
    rd = r.astype(np.float64)
    diff = hi - rd
    ulp = np.abs(np.spacing(r).astype(np.float64))
    half = ulp / 2
    tie = np.abs(diff) == half
    up = tie & (((diff > 0) & (err > 0)) | ((diff < 0) & (err < 0)))
    down = tie & (((diff > 0) & (err < 0)) | ((diff < 0) & (err > 0)))
    r = np.where(up, np.nextafter(r, np.float32(np.inf) * np.sign(diff).astype(np.float32)), r)
    r = np.where(down, r, r)
    return r.astype(np.float32)


def linspace(n):
    if n == 1:
        return np.array([-1], np.float32)
    step = f32(f32(2) / f32(n - 1))
    i = np.arange(n)
    a = fma(step, i.astype(np.float32), f32(-1))
    b = fma(-step, (n - 1 - i).astype(np.float32), f32(1))
    return np.where(i < n // 2, a, b).astype(np.float32)


def unnormalize(g, n, ac):
    if ac:
        return ((g + f32(1)) * f32(f32(n - 1) / f32(2))).astype(np.float32)
    return fma((g + f32(1)).astype(np.float32), f32(f32(n) / f32(2)), f32(-0.5))


def clip(x, n):
    return np.minimum(f32(n - 1), np.maximum(x, f32(0))).astype(np.float32)


def reflect(x, n, ac):
    if ac:
        if n <= 1:
            return np.zeros_like(x)
        ts = f32(2 * (n - 1))
        a = np.abs(x)
        flips = np.trunc((a / ts).astype(np.float32))
        extra = fma(-flips, ts, a)
        return np.minimum(extra, (ts - extra).astype(np.float32)).astype(np.float32)
    ts = f32(2 * n)
    a = np.abs((x - f32(-0.5)).astype(np.float32))
    flips = np.trunc((a / ts).astype(np.float32))
    extra = fma(-flips, ts, a)
    return (np.minimum(extra, (ts - extra).astype(np.float32)) + f32(-0.5)).astype(np.float32)


def pad_coord(x, n, pad, ac):
    if pad == "border":
        return clip(x, n)
    if pad == "reflection":
        return clip(reflect(x, n, ac), n)
    return x


def cubic(t, inner_fma=True):
    """ATen get_cubic_coefficients as compiled: the outer polynomials' products by constants are exact, so they
    read as plain; the inner ones fuse ((A+2)x - (A+3)) and the final (..)*x*x + 1."""
    A = f32(-0.75)

    def outer(x):
        return ((((A * x).astype(np.float32) - f32(5) * A) * x + f32(8) * A).astype(np.float32) * x - f32(4) * A).astype(np.float32)

    def inner(x):
        t1 = fma(f32(A + 2), x, -f32(A + 3)) if inner_fma else ((f32(A + 2) * x).astype(np.float32) - f32(A + 3)).astype(np.float32)
        return fma((t1 * x).astype(np.float32), x, f32(1))

    return (outer((t + f32(1)).astype(np.float32)), inner(t), inner((f32(1) - t).astype(np.float32)),
            outer((f32(2) - t).astype(np.float32)))


def row4(c, v, pad="zeros"):
    """x-direction sum c0 v0 + c1 v1 + c2 v2 + c3 v3 as compiled, which differs per padding instantiation:
    reflection = the same fma chain as col4; zeros / border = fma(c0, v0, c1 v1), then two plain adds."""
    if pad == "reflection":
        return col4(c, v)
    s = fma(c[0], v[0], (c[1] * v[1]).astype(np.float32))
    s = (s + (c[2] * v[2]).astype(np.float32)).astype(np.float32)
    return (s + (c[3] * v[3]).astype(np.float32)).astype(np.float32)


def col4(c, r):
    """y-direction sum: fma(c1, r1, c0 r0), then fma(c2, r2, .), fma(c3, r3, .)."""
    s = fma(c[1], r[1], (c[0] * r[0]).astype(np.float32))
    s = fma(c[2], r[2], s)
    return fma(c[3], r[3], s)


def grid_sample(img, grid, mode, pad, ac, inner_fma=True):
    """img (C, H, W) float32, grid (Ho, Wo, 2) float32 -> (C, Ho, Wo)."""
    C, H, W = img.shape
    gx, gy = grid[..., 0], grid[..., 1]

    def tap(c, x, y):
        ok = (x >= 0) & (x < W) & (y >= 0) & (y < H)
        return np.where(ok, img[c][np.clip(y, 0, H - 1), np.clip(x, 0, W - 1)], f32(0)).astype(np.float32)

    out = np.zeros((C,) + gx.shape, np.float32)
    if mode == "bicubic":
        x = unnormalize(gx, W, ac)
        y = unnormalize(gy, H, ac)
        fx, fy = np.floor(x), np.floor(y)
        cx, cy = cubic((x - fx).astype(np.float32), inner_fma), cubic((y - fy).astype(np.float32), inner_fma)

        def bounded(c, xx, yy):
            xx = pad_coord(xx, W, pad, ac)
            yy = pad_coord(yy, H, pad, ac)
            return tap(c, xx.astype(np.int64), yy.astype(np.int64))

        for c in range(C):
            rows = []
            for i in range(4):
                yy = (fy + f32(-1 + i)).astype(np.float32)
                v = [bounded(c, (fx + f32(-1 + j)).astype(np.float32), yy) for j in range(4)]
                rows.append(row4(cx, v, pad))
            out[c] = col4(cy, rows)
        return out
    x = pad_coord(unnormalize(gx, W, ac), W, pad, ac)
    y = pad_coord(unnormalize(gy, H, ac), H, pad, ac)
    if mode == "nearest":
        xn, yn = np.rint(x), np.rint(y)
        for c in range(C):
            out[c] = tap(c, xn.astype(np.int64), yn.astype(np.int64))
        return out
    fx, fy = np.floor(x), np.floor(y)
    w = (x - fx).astype(np.float32)
    e = (f32(1) - w).astype(np.float32)
    n_ = (y - fy).astype(np.float32)
    s = (f32(1) - n_).astype(np.float32)
    nw, ne, sw, se = (s * e).astype(np.float32), (s * w).astype(np.float32), (n_ * e).astype(np.float32), (n_ * w).astype(np.float32)
    x0, y0 = fx.astype(np.int64), fy.astype(np.int64)
    for c in range(C):
        v0, v1, v2, v3 = tap(c, x0, y0), tap(c, x0 + 1, y0), tap(c, x0, y0 + 1), tap(c, x0 + 1, y0 + 1)
        out[c] = fma(v3, se, fma(v2, sw, fma(v1, ne, (v0 * nw).astype(np.float32))))
    return out


def main():
    g = torch.Generator().manual_seed(0)
    bad_total = 0
    for n in (7, 109, 256, 436, 1024, 1242):
        bad = int((linspace(n) != torch.linspace(-1, 1, n).numpy()).sum())
        bad_total += bad
        print(f"linspace {n}: {bad} mismatches")
    for (H, W) in ((13, 17), (40, 64)):
        img = torch.rand(2, H, W, generator=g) * 255
        for scale in (1.1, 3.0):
            grid = torch.rand(40, 50, 2, generator=g) * 2 * scale - scale
            grid[0, 0] = torch.tensor([1.0, -1.0])
            grid[0, 1] = torch.tensor([0.5 / W * 2 - 1, 0.5 / H * 2 - 1])
            for mode in ("bilinear", "nearest", "bicubic"):
                for pad in ("zeros", "border", "reflection"):
                    for ac in (False, True):
                        ref = F.grid_sample(img[None], grid[None], mode, pad, ac)[0].numpy()
                        got = grid_sample(img.numpy(), grid.numpy(), mode, pad, ac)
                        bad = int((ref != got).sum())
                        if mode == "bicubic":
                            alt = int((ref != grid_sample(img.numpy(), grid.numpy(), mode, pad, ac, False)).sum())
                            if alt != bad:
                                print("inner fma", bad, "vs plain", alt, pad, ac)
                        bad_total += bad
                        if bad:
                            print(H, W, scale, mode, pad, ac, bad, float(np.abs(ref - got).max()))
    print("total mismatches", bad_total)


if __name__ == "__main__":
    main()
