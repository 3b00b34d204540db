"""EXPERIMENT driver: the product lookup kernels vs the round-1 ones (tools/exp/lookup_r01.hip), same pyramid and
coords, interleaved rounds in one process (cdna_hip_programming.md §5.4 rule 24). Each launch is bracketed by its own
event pair on the stream, with no host sync in between (the queue stays ahead): 'hot' = back-to-back launches (the
~170 MB of window lines stay in the 256 MiB Infinity Cache), 'cold' = a 1 GiB buffer is read before every launch."""
import ctypes
import json
import os
import statistics
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
PKG = os.path.join(REPO, "torch-optical-flow_amd")
for p in (REPO, PKG, os.path.join(PKG, "methods", "raft")):
    sys.path.insert(0, p)

import torch  # noqa: E402

from bench import lookup_bytes  # noqa: E402
from model import synthetic  # noqa: E402
from model.utils import coords_grid  # noqa: E402
from optical_flow import _native  # noqa: E402

SO = os.path.join(HERE, "liblookup_r01.so")
if not os.path.exists(SO):
    subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-shared", "-fPIC",
                    "-I" + os.path.join(REPO, "include"), "-o", SO, os.path.join(HERE, "lookup_r01.hip")], check=True)
lib = ctypes.CDLL(SO)
VP, I = ctypes.c_void_p, ctypes.c_int
SHAPES = {"sintel8": (8, 55, 128), "corr4": (4, 128, 128), "kitti8": (8, 47, 156)}


def timed(fn, n, flush=None):
    evs = []
    for _ in range(n):
        if flush is not None:
            flush()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        evs.append((a, b))
    torch.cuda.synchronize()
    return statistics.median(a.elapsed_time(b) for a, b in evs) * 1e3  # us


def main():
    shape = sys.argv[1] if len(sys.argv) > 1 else "sintel8"
    b, h, w = SHAPES[shape]
    dev = torch.device("cuda", 0)
    f1, f2 = synthetic.synthetic_fmaps(b, 256, h, w, stream=3)
    f1, f2 = f1.to(dev), f2.to(dev)
    coords = (coords_grid(b, h, w) + torch.from_numpy(synthetic.hash_normal(4, (b, 2, h, w), 4.0))).to(dev)
    tp = _native.corr_pyramid_tiled(f1, f2, 4)
    dims = tp.dims
    nb = lookup_bytes(b, dims)
    scratch = torch.ones(1 << 28, device=dev)
    flush = lambda: scratch.sum()  # noqa: E731
    ptrs = (VP * 4)(*[t.data_ptr() for t in tp.levels])
    hs = (I * 4)(*[d[0] for d in dims])
    ws = (I * 4)(*[d[1] for d in dims])
    st = VP(torch.cuda.current_stream().cuda_stream)
    out_nchw = torch.empty((b, 324, h, w), device=dev)
    rows352 = torch.empty((b * h * w, 352), device=dev)
    rows324 = torch.empty((b * h * w, 324), device=dev)
    variants = {
        "r01_nchw": lambda: lib.r01_corr_lookup_tiled_f32(ptrs, hs, ws, 4, VP(coords.data_ptr()), b, h, w, 4, VP(out_nchw.data_ptr()), st),
        "r01_nhwc352": lambda: lib.r01_corr_lookup_tiled_nhwc_f32(ptrs, hs, ws, 4, VP(coords.data_ptr()), b, h, w, 4, VP(rows352.data_ptr()), 352, st),
        "new_nchw": lambda: _native.corr_lookup_tiled(tp, coords, 4),
        "new_nhwc324": lambda: _native.corr_lookup_tiled_nhwc(tp, coords, 4, rows324),
    }
    res = {k: {"hot": [], "cold": []} for k in variants}
    for _ in range(3):
        for k, fn in variants.items():
            res[k]["hot"].append(timed(fn, 30))
            res[k]["cold"].append(timed(fn, 15, flush))
    out = {"shape": shape, "algorithmic_bytes": nb}
    for k, v in res.items():
        hot, cold = statistics.median(v["hot"]), statistics.median(v["cold"])
        out[k] = {"hot_us": round(hot, 2), "cold_us": round(cold, 2), "cold_frac": round(nb / (cold * 1e-6) / 8e12, 4)}
    ref = _native.corr_lookup_tiled(tp, coords, 4)
    variants["r01_nchw"]()
    torch.cuda.synchronize()
    out["r01_equals_new"] = bool(torch.equal(ref, out_nchw))
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
