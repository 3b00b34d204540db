"""EXPERIMENT driver: ablations of the product conv_s32 kernel (conv_abl.hip ABL bits) at the update-block shapes,
interleaved rounds in one process; ABL 0 must equal the product bit for bit."""
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

lib = ctypes.CDLL(os.path.join(HERE, "libconv_abl.so"))
real = N.load()
lib.exp_conv_abl.restype = ctypes.c_int
lib.exp_conv_abl.argtypes = [ctypes.c_int] + list(real.oflow_conv_s32_ex.argtypes)
ABLS = [int(v) for v in os.environ.get("ABLS", "0,1,2,4,8,16,25,27").split(",")]


class Proxy:
    abl = -1

    def __getattr__(self, k):
        if k == "oflow_conv_s32_ex2" and Proxy.abl >= 0:
            return lambda *a: lib.exp_conv_abl(Proxy.abl, *a[:-4], a[-1])
        return getattr(real, k)


N._lib = Proxy()


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


def main():
    b, h, w = 8, 55, 128
    dev = torch.device("cuda", 0)
    P = b * h * w
    g = torch.Generator().manual_seed(0)
    hm = torch.randn(P, 128, device=dev)
    z = torch.rand(P, 128, device=dev)
    layers = [
        ("convc1 1x1 352->256", 1, 1, 352, 256, 256, 128, 11, 8, 0),
        ("convc2 3x3 256->192", 3, 3, 256, 192, 192, 64, 8, 6, 0),
        ("conv 3x3 256->126", 3, 3, 256, 126, 128, 128, 8, 4, 0),
        ("gru zr 1x5 384->256", 1, 5, 384, 256, 256, 128, 12, 4, 1),
        ("gru q 5x1 384->128", 5, 1, 384, 128, 128, 128, 12, 4, 2),
    ]
    res = {}
    for name, kh, kw, cin, n, npad, bn, gi, go, epi in layers:
        x = N.s32_from_f32(torch.randn(b, gi * 32, h, w, generator=g).to(dev))
        wt = (torch.randn(n, cin, kh, kw, generator=g) * 0.03).to(dev)
        cw = N.ConvWeights(wt, torch.zeros(n, device=dev), npad)
        outs = {}
        for v in [-1] + ABLS:
            if epi:
                y = N.s32_empty(b, h, w, 4, dev, zero=True)
                kw_ = dict(epilogue=epi, y0=N.S32Slice(y), gru_h=hm.clone(), gru_z=z.clone())
            else:
                y = N.s32_empty(b, h, w, go, dev, zero=True)
                kw_ = dict(act="relu", y0=N.S32Slice(y))
            Proxy.abl = v
            N.conv_s32(N.S32Slice(x), cw, bn, **kw_)
            torch.cuda.synchronize()
            outs[v] = (y.clone(), kw_)
        eq0 = bool(torch.equal(outs[0][0], outs[-1][0]))
        times = {v: [] for v in [-1] + ABLS}
        for _ in range(5):
            for v in [-1] + ABLS:
                Proxy.abl = v
                kw_ = outs[v][1]
                times[v].append(timed(lambda: N.conv_s32(N.S32Slice(x), cw, bn, **kw_), 20) * 1e3)
        res[name] = {"abl0_equals_product": eq0, **{str(v): round(statistics.median(t), 1) for v, t in times.items()}}
        print(name, res[name], flush=True)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
