"""Micro-bench of the split-fp16 update-block kernels at RAFT shapes (HIP-event timed, back-to-back launches).

Prints, per layer of one update iteration: us per launch, the fp32-equivalent TFLOP/s (2*M*N*K of the real conv)
and the fraction of the fp16 MFMA peak the 3 split products use (3 x padded flops / 2.5 PF). Also the S32 lookup.

    python tools/convbench.py [--shape sintel8|kitti8] [--iters 30]
"""
import argparse
import json
import os
import statistics
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(REPO, "torch-optical-flow_amd")
for p in (REPO, PKG, os.path.join(PKG, "methods", "raft")):
    sys.path.insert(0, p)

import torch  # noqa: E402

from bench import lookup_bytes  # noqa: E402
from model import synthetic  # noqa: E402
from model.utils import coords_grid  # noqa: E402
from optical_flow import _native as N  # noqa: E402

SHAPES = {"sintel8": (8, 55, 128), "kitti8": (8, 47, 156)}
F16_PEAK = 2.5e15


def timed(fn, n):
    fn()
    torch.cuda.synchronize()
    rounds = []
    for _ in range(3):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(n):
            fn()
        b.record()
        b.synchronize()
        rounds.append(a.elapsed_time(b) / n)
    return statistics.median(rounds)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shape", default="sintel8", choices=sorted(SHAPES))
    ap.add_argument("--iters", type=int, default=30)
    ap.add_argument("--layer", default=None, help="only layers whose name contains this string (PMC runs)")
    ap.add_argument("--no-lookup", action="store_true")
    ap.add_argument("--ablate", action="store_true", help="with the -DOFLOW_ABLATE library build (OFLOW_LIB): per-layer "
                    "times with kernel parts dropped (exp_flags: 2 MFMAs, 4 A staging, 16 epilogue, 32 B staging, "
                    "64 main-loop barriers)")
    ap.add_argument("--shape-batch", type=int, default=0, help="override the batch (pairs) of --shape")
    ap.add_argument("--conv-flags", type=int, default=0, help="oflow_exp_set_conv_flags value for the run (experiments)")
    args = ap.parse_args()
    if args.conv_flags:
        N.load().oflow_exp_set_conv_flags(args.conv_flags)
    b, h, w = SHAPES[args.shape]
    if args.shape_batch:
        b = args.shape_batch
    dev = torch.device("cuda", 0)
    P = b * h * w
    g = torch.Generator().manual_seed(0)

    def s32(groups):
        x = torch.randn(b, groups * 32, h, w, generator=g).to(dev)
        return N.s32_from_f32(x)

    def weights(n, cin, kh, kw, npad):
        wt = (torch.randn(n, cin, kh, kw, generator=g) * 0.03).to(dev)
        return N.ConvWeights(wt, torch.zeros(n, device=dev), npad)

    hm = torch.randn(P, 128, device=dev)
    z = torch.rand(P, 128, device=dev)
    layers = [
        # name, kh, kw, cin, n, npad, block_n, in groups, out groups, epilogue
        ("convc1 1x1 352->256", 1, 1, 352, 256, 256, 128, 11, 8, 0),
        ("convc2 3x3 256->192", 3, 3, 256, 192, 192, 64, 8, 6, 0),
        ("convf1 1x1 128->128", 1, 1, 128, 128, 128, 128, 4, 4, 0),
        ("convf2 3x3 128->64", 3, 3, 128, 64, 64, 64, 4, 2, 0),
        ("conv 3x3 256->126", 3, 3, 256, 126, 128, 128, 8, 4, 0),
        # the GRU convs contract [h | motion | flow] (8 groups); the context term W_inp*inp + b comes as the addend
        ("gru zr 1x5 256->256", 1, 5, 256, 256, 256, 128, 8, 4, 1),
        ("gru q 1x5 256->128", 1, 5, 256, 128, 128, 128, 8, 4, 2),
        ("gru zr 5x1 256->256", 5, 1, 256, 256, 256, 128, 8, 4, 1),
        ("gru q 5x1 256->128", 5, 1, 256, 128, 128, 128, 8, 4, 2),
        ("fh1 3x3 128->256", 3, 3, 128, 256, 256, 128, 4, 8, 0),
        ("fh2 3x3 256->2", 3, 3, 256, 2, 32, 32, 8, 0, 0),
    ]
    out = {"shape": args.shape, "layers": {}}
    total = 0.0
    for name, kh, kw, cin, n, npad, bn, gi, go, epi in layers:
        if args.layer and args.layer not in name:
            continue
        x = s32(gi)
        cw = weights(n, cin, kh, kw, npad)
        kw_ = {}
        if epi:
            kw_ = dict(epilogue=epi, y0=N.S32Slice(N.s32_empty(b, h, w, 4, dev)), gru_h=hm, gru_z=z,
                       addend=torch.randn(P, n, device=dev))
        elif go:
            kw_ = dict(act="relu", y0=N.S32Slice(N.s32_empty(b, h, w, go, dev)))
        else:
            kw_ = dict(f32=torch.zeros(b, 2, h, w, device=dev), f32_accumulate=True)
        ms = timed(lambda: N.conv_s32(N.S32Slice(x), cw, bn, **kw_), args.iters)
        total += ms
        if args.ablate:  # the -DOFLOW_ABLATE library: time with parts of the kernel dropped
            lib = N.load()
            abl = {}
            for f in (2, 4, 16, 32, 64, 2 | 4 | 32, 2 | 4 | 16 | 32 | 64):
                lib.oflow_exp_set_conv_flags(f)
                abl[str(f)] = round(timed(lambda: N.conv_s32(N.S32Slice(x), cw, bn, **kw_), args.iters) * 1e3, 1)
            lib.oflow_exp_set_conv_flags(0)
        flops = 2.0 * P * n * cin * kh * kw
        padded = 2.0 * P * npad * (gi * 32) * kh * kw * 3
        out["layers"][name] = {
            "us": round(ms * 1e3, 1),
            "tflops_f32_equiv": round(flops / ms / 1e9, 1),
            "mfma_frac": round(padded / (ms * 1e-3) / F16_PEAK, 3),
        }
        if args.ablate:
            out["layers"][name]["ablated_us"] = abl
    out["update_iteration_convs_us"] = round(total * 1e3, 1)
    if args.no_lookup:
        print(json.dumps(out, indent=1))
        return
    # the lookup (NHWC rows and NCHW) on a real pyramid
    f1, f2 = synthetic.synthetic_fmaps(b, 256, h, w, stream=3)
    f1, f2 = f1.to(dev), f2.to(dev)
    coords = (coords_grid(b, h, w) + torch.from_numpy(synthetic.hash_normal(4, (b, 2, h, w), 4.0))).to(dev)
    tp = N.corr_pyramid_tiled(f1, f2, 4)
    dims = tp.dims
    lf = torch.empty((b * h * w, 324), device=dev)
    lnh = timed(lambda: N.corr_lookup_tiled_nhwc(tp, coords, 4, lf), args.iters * 3)
    ln = timed(lambda: N.corr_lookup_tiled(tp, coords, 4), args.iters * 3)
    lb = lookup_bytes(b, dims)
    out["lookup_nhwc_us"] = round(lnh * 1e3, 1)
    out["lookup_nhwc_GBs"] = round(lb / lnh / 1e6, 1)
    out["lookup_nchw_us"] = round(ln * 1e3, 1)
    out["lookup_nchw_GBs"] = round(lb / ln / 1e6, 1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
