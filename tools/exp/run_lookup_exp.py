"""EXPERIMENT driver: time lookup variants on blocked layouts vs the product kernel (same inputs, same outputs)."""
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

from model import synthetic  # noqa: E402
from model.utils import coords_grid  # noqa: E402
from optical_flow import _native  # noqa: E402
from bench import lookup_bytes  # noqa: E402

SO = os.path.join(HERE, "liblookup_exp.so")
if not os.path.exists(SO):
    subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-shared", "-fPIC", "-o", SO, os.path.join(HERE, "lookup_exp.hip")], check=True)
lib = ctypes.CDLL(SO)
VP = ctypes.c_void_p


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

def run(shape, b, h, w, sigma):
    dev = torch.device("cuda", 0)
    f1, f2 = synthetic.synthetic_fmaps(b, 256, h, w, stream=3)
    pyr = _native.corr_pyramid(f1.to(dev), f2.to(dev), 4)
    coords = (coords_grid(b, h, w) + torch.from_numpy(synthetic.hash_normal(4, (b, 2, h, w), sigma))).to(dev)
    ref = _native.corr_lookup(pyr, coords, 4)
    dims = [(int(p.shape[2]), int(p.shape[3])) for p in pyr]
    nbytes = lookup_bytes(b, dims)
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    res = {"shape": shape, "sigma": sigma}
    t = timed(lambda: _native.corr_lookup(pyr, coords, 4))
    res["product"] = (round(t * 1e3, 1), round(nbytes / t / 1e6))
    q = b * h * w
    lvp = (VP * 4)(*[p.data_ptr() for p in pyr])
    hs0 = (ctypes.c_int * 4)(*[d[0] for d in dims])
    ws0 = (ctypes.c_int * 4)(*[d[1] for d in dims])
    for mode, qpb in [(0, 64), (1, 64), (2, 64), (3, 64), (4, 64), (0, 32), (0, 16), (1, 32), (3, 32)]:
        out = torch.empty_like(ref)
        def go():
            assert lib.exp_lookup_ablate(lvp, hs0, ws0, mode, qpb, VP(coords.data_ptr()), b, h * w, VP(out.data_ptr()), st) == 0
        go()
        torch.cuda.synchronize()
        err = float((out - ref).abs().max()) if mode == 0 else None
        t = timed(go)
        res[f"ablate_m{mode}_q{qpb}"] = (round(t * 1e3, 1), err)
    for bh, bw, mode in [(4, 4, 0), (4, 8, 0), (8, 4, 0), (4, 4, 4), (4, 8, 4), (8, 8, 0), (2, 8, 0)]:
        blk = []
        for p, (hl, wl) in zip(pyr, dims):
            hb, wb = -(-hl // bh), -(-wl // bw)
            o = torch.empty(q * hb * wb * bh * bw, device=dev)
            assert lib.exp_relayout(VP(p.data_ptr()), VP(o.data_ptr()), ctypes.c_longlong(q), hl, wl, bh, bw, st) == 0
            blk.append(o)
        out = torch.empty_like(ref)
        ptrs = (VP * 4)(*[x.data_ptr() for x in blk])
        def go():
            assert lib.exp_lookup_hybrid(ptrs, hs0, ws0, bh, bw, mode, VP(coords.data_ptr()), b, h * w, VP(out.data_ptr()), st) == 0
        go()
        torch.cuda.synchronize()
        err = float((out - ref).abs().max()) if mode == 0 else None
        t = timed(go)
        res[f"hybrid{bh}x{bw}m{mode}"] = (round(t * 1e3, 1), round(nbytes / t / 1e6), err)
        del blk
    for bh, bw, qpb in [(4, 4, 32)]:
        blk = []
        for p, (hl, wl) in zip(pyr, dims):
            hb, wb = -(-hl // bh), -(-wl // bw)
            o = torch.empty(q * hb * wb * bh * bw, device=dev)
            assert lib.exp_relayout(VP(p.data_ptr()), VP(o.data_ptr()), ctypes.c_longlong(q), hl, wl, bh, bw, st) == 0
            blk.append(o)
        out = torch.empty_like(ref)
        ptrs = (VP * 4)(*[x.data_ptr() for x in blk])
        hs = (ctypes.c_int * 4)(*[d[0] for d in dims])
        ws = (ctypes.c_int * 4)(*[d[1] for d in dims])

        def go():
            assert lib.exp_lookup_blocked(ptrs, hs, ws, bh, bw, qpb, VP(coords.data_ptr()), b, h * w, VP(out.data_ptr()), st) == 0

        go()
        torch.cuda.synchronize()
        err = float((out - ref).abs().max())
        t = timed(go)
        res[f"blk{bh}x{bw}q{qpb}"] = (round(t * 1e3, 1), round(nbytes / t / 1e6), err)
        del blk
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    run("sintel8", 8, 55, 128, 4.0)
    run("sintel8_s0", 8, 55, 128, 0.0)
    run("corr4", 4, 128, 128, 4.0)
    run("kitti8", 8, 47, 156, 4.0)
