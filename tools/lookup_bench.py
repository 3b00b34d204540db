"""Lookup kernel bench at the bench workload's shape: both output forms of the segment-DMA lookup, hot (back-to-back
launches: the ~170 MB of lines one lookup touches stay in the 256 MiB Infinity Cache) and cold (a 1 GiB buffer is
read between launches so every line comes from HBM, as inside the RAFT step), each launch timed by its own HIP
event pair on the launch stream.

    python tools/lookup_bench.py [--shape sintel8|kitti8|corr4] [--sigma 4] [--iters 20]
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
from optical_flow import _native  # noqa: E402

SHAPES = {"sintel8": (8, 55, 128), "corr4": (4, 128, 128), "kitti8": (8, 47, 156), "sintel1": (1, 55, 128)}


def per_launch(fn, n, flush=None):
    """Median of n individually event-timed launches (flush() runs before each one, outside its events)."""
    ts = []
    fn()
    for _ in range(n):
        if flush is not None:
            flush()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        b.synchronize()
        ts.append(a.elapsed_time(b))
    return statistics.median(ts), min(ts)


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
    tp = _native.corr_pyramid_tiled(f1, f2, 4)
    dims = tp.dims
    scratch = torch.ones(1 << 28, device=dev)  # 1 GiB, read (not written) between launches: evicts without dirty lines
    flush = lambda: scratch.sum()  # noqa: E731
    rows = torch.empty((b * h * w, 4 * 81), device=dev)
    res = {"shape": args.shape, "sigma": args.sigma, "algorithmic_bytes": lookup_bytes(b, dims)}
    for name, fn in (
        ("nhwc", lambda: _native.corr_lookup_tiled_nhwc(tp, coords, 4, rows)),
        ("nchw", lambda: _native.corr_lookup_tiled(tp, coords, 4)),
    ):
        for mode, fl in (("hot", None), ("cold", flush)):
            med, best = per_launch(fn, args.iters, fl)
            res[f"{name}_{mode}_us"] = round(med * 1e3, 2)
            res[f"{name}_{mode}_frac"] = round(res["algorithmic_bytes"] / (med * 1e-3) / 8e12, 4)
    # correctness spot check: NHWC rows == NCHW permuted
    ref = _native.corr_lookup_tiled(tp, coords, 4)
    _native.corr_lookup_tiled_nhwc(tp, coords, 4, rows)
    res["nhwc_equals_nchw"] = bool(torch.equal(rows.view(b, h, w, -1), ref.permute(0, 2, 3, 1)))
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
