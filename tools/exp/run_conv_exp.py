"""EXPERIMENT driver: the update-block convs (tools/convbench.py shapes) with conv_s32 schedule variants (VAR hooks),
interleaved rounds in one process; outputs checked bit-equal to VAR 0."""
import ctypes
import json
import os
import statistics
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
PKG = os.path.join(REPO, "torch-optical-flow_amd")
for p in (REPO, PKG, os.path.join(PKG, "methods", "raft")):
    sys.path.insert(0, p)

import torch  # noqa: E402

from optical_flow import _native as N  # noqa: E402

exp = ctypes.CDLL(os.path.join(HERE, os.environ.get("EXP_LIB", "libconv_exp.so")))
real = N.load()
exp.exp_conv_s32_var.restype = ctypes.c_int
exp.exp_conv_s32_var.argtypes = [ctypes.c_int] + list(real.oflow_conv_s32_ex.argtypes)


class Proxy:
    var = 0

    def __getattr__(self, k):
        if k == "oflow_conv_s32_ex2":  # the product wrapper's entry: S32 inputs only here (last 3 args in_format..)
            if Proxy.var < 0:  # VAR -1: the current product kernel
                return real.oflow_conv_s32_ex2
            return lambda *a: exp.exp_conv_s32_var(Proxy.var, *a[:-4], a[-1])
        return getattr(real, k)


N._lib = Proxy()
VARS = [int(v) for v in os.environ.get("VARS", "0,1,2,3,4,6").split(",")]


def timed(fn, n):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(n):
        fn()
    b.record()
    b.synchronize()
    return a.elapsed_time(b) / n


def batch_scan():
    """zr 1x5 at several batch sizes (workgroup-count quantization vs 2 workgroups per CU x 256 CUs)."""
    dev = torch.device("cuda", 0)
    g = torch.Generator().manual_seed(0)
    wt = (torch.randn(256, 384, 1, 5, generator=g) * 0.03).to(dev)
    cw = N.ConvWeights(wt, torch.zeros(256, device=dev), 256)
    out = {}
    for b in (1, 2, 4, 6, 8, 9, 10, 12, 16):
        h, w = 55, 128
        x = N.s32_from_f32(torch.randn(b, 384, h, w, generator=g).to(dev))
        P = b * h * w
        kw_ = dict(epilogue=1, y0=N.S32Slice(N.s32_empty(b, h, w, 4, dev)), gru_h=torch.randn(P, 128, device=dev),
                   gru_z=torch.rand(P, 128, device=dev))
        Proxy.var = 0
        t = statistics.median(timed(lambda: N.conv_s32(N.S32Slice(x), cw, 128, **kw_), 10) for _ in range(3))
        wgs = 4 * 14 * b * 2
        out[b] = {"us": round(t * 1e3, 1), "us_per_pair": round(t * 1e3 / b, 1), "workgroups": wgs,
                  "generations": round(wgs / 512, 3)}
        print("zr batch", b, out[b], flush=True)
    return out


def main():
    if os.environ.get("BATCH_SCAN"):
        print(json.dumps(batch_scan()))
        return
    b, h, w = 8, 55, 128
    dev = torch.device("cuda", 0)
    P = b * h * w
    g = torch.Generator().manual_seed(0)

    def s32(groups, bb=b, hh=h, ww=w):
        x = torch.randn(bb, groups * 32, hh, ww, generator=g).to(dev)
        return N.s32_from_f32(x)

    def weights(n, cin, kh, kw, npad):
        wt = (torch.randn(n, cin, kh, kw, generator=g) * 0.03).to(dev)
        return N.ConvWeights(wt, torch.zeros(n, device=dev), npad)

    hm = torch.randn(P, 128, device=dev)
    z = torch.rand(P, 128, device=dev)
    layers = [
        ("convc1 1x1 352->256", 1, 1, 352, 256, 256, 128, 11, 8, 0),
        ("convc2 3x3 256->192", 3, 3, 256, 192, 192, 64, 8, 6, 0),
        ("conv 3x3 256->126", 3, 3, 256, 126, 128, 128, 8, 4, 0),
        ("gru zr 1x5 384->256", 1, 5, 384, 256, 256, 128, 12, 4, 1),
        ("gru q 5x1 384->128", 5, 1, 384, 128, 128, 128, 12, 4, 2),
        ("fh1 3x3 128->256", 3, 3, 128, 256, 256, 128, 4, 8, 0),
    ]
    res = {}
    for name, kh, kw, cin, n, npad, bn, gi, go, epi in layers:
        x = s32(gi)
        cw = weights(n, cin, kh, kw, npad)
        outs = {}
        for v in VARS:
            if epi:
                hcopy = hm.clone()
                y = N.s32_empty(b, h, w, 4, dev, zero=True)
                kw_ = dict(epilogue=epi, y0=N.S32Slice(y), gru_h=hcopy, gru_z=z.clone())
            else:
                y = N.s32_empty(b, h, w, go, dev, zero=True)
                kw_ = dict(act="relu", y0=N.S32Slice(y))
            Proxy.var = v
            N.conv_s32(N.S32Slice(x), cw, bn, **kw_)
            torch.cuda.synchronize()
            outs[v] = (y.clone(), kw_)
        eq = {v: bool(torch.equal(outs[v][0], outs[VARS[0]][0])) for v in VARS}  # ablations (VAR >= 128) differ
        times = {v: [] for v in VARS}
        for _ in range(5):
            for v in VARS:
                Proxy.var = v
                kw_ = outs[v][1]
                times[v].append(timed(lambda: N.conv_s32(N.S32Slice(x), cw, bn, **kw_), 20) * 1e3)
        res[name] = {str(v): (round(statistics.median(t), 1), round(min(t), 1), eq[v]) for v, t in times.items()}
        print(name, res[name], flush=True)
    # encoder layer1 shape (fnet: 16 images at 220x512, 64 -> 64 3x3): epilogue ablation at VAR 0
    bb, hh, ww = 16, 220, 512
    x = s32(2, bb, hh, ww)
    cw = weights(64, 64, 3, 3, 64)
    raw = torch.empty((bb * hh * ww, 64), device=dev)
    part = torch.empty((bb, N.conv_tiles(hh, ww), 64, 3), device=dev)
    ys = N.s32_empty(bb, hh, ww, 2, dev)
    cases = {
        "nhwc+stats": dict(nhwc=raw, stats=part),
        "nhwc": dict(nhwc=raw),
        "stats": dict(stats=part),
        "s32": dict(y0=N.S32Slice(ys)),
    }
    times = {(k, v): [] for k in cases for v in VARS}
    for _ in range(3):
        for k, kw_ in cases.items():
            for v in VARS:
                Proxy.var = v
                times[(k, v)].append(timed(lambda: N.conv_s32(N.S32Slice(x), cw, 64, **kw_), 5) * 1e3)
    res["enc l1 3x3 64 epilogues"] = {f"{k}/{v}": round(statistics.median(t), 1) for (k, v), t in times.items()}
    # and the same conv at BN 64 with 32-px-wide tiles vs a 3x3 128 -> 128 (layer-3-like) shape
    print(res["enc l1 3x3 64 epilogues"], flush=True)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
