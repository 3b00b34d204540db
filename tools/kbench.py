"""Kernel micro-bench: corr_pyramid and corr_lookup alone at BASELINE shapes, HIP-event timed (median of N).

    python tools/kbench.py [--shape sintel8|corr4|kitti8|hd1] [--iters 20]
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

from bench import lookup_bytes, pyramid_cost  # noqa: E402
from model import synthetic  # noqa: E402
from model.utils import coords_grid  # noqa: E402
from optical_flow import _native  # noqa: E402

SHAPES = {"sintel8": (8, 55, 128), "corr4": (4, 128, 128), "kitti8": (8, 47, 156), "sintel1": (1, 55, 128), "hd1": (1, 135, 240)}


def timed(fn, n=50):
    """Mean per-launch time of n back-to-back launches between one event pair (median of 3 rounds): the queue
    stays ahead of the GPU, so host launch latency is not in the number."""
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
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--sigma", type=float, default=4.0)
    args = ap.parse_args()
    b, h, w = SHAPES[args.shape]
    dev = torch.device("cuda", 0)
    f1, f2 = synthetic.synthetic_fmaps(b, 256, h, w, stream=3)
    f1, f2 = f1.to(dev), f2.to(dev)
    coords = (coords_grid(b, h, w) + torch.from_numpy(synthetic.hash_normal(4, (b, 2, h, w), args.sigma))).to(dev)
    pyr = _native.corr_pyramid(f1, f2, 4)
    torch.cuda.synchronize()
    dims = [(int(p.shape[2]), int(p.shape[3])) for p in pyr]
    del pyr
    torch.cuda.empty_cache()
    pm = timed(lambda: _native.corr_pyramid(f1, f2, 4), args.iters)
    s1, s2 = _native.s32_from_f32(f1), _native.s32_from_f32(f2)
    pms = timed(lambda: _native.corr_pyramid_tiled_s32(s1, s2, 4), args.iters)  # the RAFT forward's split-fp16 build
    del s1, s2
    pyr = _native.corr_pyramid(f1, f2, 4)
    lm_canon = timed(lambda: _native.corr_lookup(pyr, coords, 4), args.iters * 5)
    del pyr
    torch.cuda.empty_cache()
    pmt = timed(lambda: _native.corr_pyramid_tiled(f1, f2, 4), args.iters)
    tp = _native.corr_pyramid_tiled(f1, f2, 4)
    lm = timed(lambda: _native.corr_lookup_tiled(tp, coords, 4), args.iters * 5)
    # warp operator at the SURVEY §8(d) shape: frame (8, 3, 436, 1024), flow = normalize(N(0, 8^2) px)
    import optical_flow
    frame, _ = synthetic.synthetic_pair(8, 436, 1024, seed=1)
    flow = optical_flow.normalize(torch.from_numpy(synthetic.hash_normal(5, (8, 2, 436, 1024), 8.0)))
    frame, flow = frame.to(dev), flow.to(dev)
    wm = timed(lambda: optical_flow.warp(frame, flow), args.iters * 5)
    wbytes = (2 * 3 + 2) * 4 * 8 * 436 * 1024
    flops, pbytes = pyramid_cost(b, dims)
    lb = lookup_bytes(b, dims)
    print(
        json.dumps(
            {
                "shape": args.shape,
                "pyramid_s32_ms": round(pms, 5),
                "pyramid_s32_f16_tflops": round(3 * pyramid_cost(b, dims)[0] / pms / 1e9, 2),
                "pyramid_ms": round(pm, 4),
                "pyramid_tflops": round(flops / pm / 1e9, 2),
                "pyramid_GBs": round(pbytes / pm / 1e6, 1),
                "pyramid_tiled_ms": round(pmt, 4),
                "lookup_ms": round(lm, 5),
                "lookup_canonical_ms": round(lm_canon, 5),
                "lookup_canonical_GBs": round(lb / lm_canon / 1e6, 1),
                "lookup_GBs": round(lb / lm / 1e6, 1),
                "lookup_bytes": lb,
                "warp_ms": round(wm, 5),
                "warp_GBs": round(wbytes / wm / 1e6, 1),
            }
        )
    )


if __name__ == "__main__":
    main()
