"""EXPERIMENT: how fast can the memory system deliver exactly the 128-B lines one Sintel x8 lookup touches?
Builds the line list from the same pyramid geometry and coords as the lookup (tiled 4x8 layout, windows clipped to
the level), then times (a) a fully coalesced gather of those lines, (b) a 16-B stream write of the lookup's output
bytes, (c) the product NHWC lookup -- each cold (1 GiB read before every launch), event-timed, median of 15."""
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

SO = os.path.join(HERE, "libline_gather.so")
if not os.path.exists(SO):
    subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-shared", "-fPIC", "-o", SO,
                    os.path.join(HERE, "line_gather.hip")], check=True)
lib = ctypes.CDLL(SO)
VP = ctypes.c_void_p


def window_lines(tp, coords, radius=4):
    """Sorted-by-query int64 line indices (units of 128 B from level 0's base) of every tile a window touches."""
    b, _, h, w = coords.shape
    q = b * h * w
    base0 = tp.levels[0].data_ptr()
    out = []
    cx = coords[:, 0].reshape(-1)
    cy = coords[:, 1].reshape(-1)
    qi = torch.arange(q, device=coords.device)
    for l, (hl, wl) in enumerate(tp.dims):
        hb, wb = (hl + 3) // 4, (wl + 7) // 8
        lbase = (tp.levels[l].data_ptr() - base0) // 128
        xs = torch.floor(cx / 2 ** l).long() - radius
        ys = torch.floor(cy / 2 ** l).long() - radius
        pk = 2 * radius + 2
        x0, x1 = xs.clamp(0, wl - 1), (xs + pk - 1).clamp(0, wl - 1)
        y0, y1 = ys.clamp(0, hl - 1), (ys + pk - 1).clamp(0, hl - 1)
        valid = (xs + pk - 1 >= 0) & (xs < wl) & (ys + pk - 1 >= 0) & (ys < hl)
        for dty in range(4):
            for dtx in range(3):
                ty = y0 // 4 + dty
                tx = x0 // 8 + dtx
                m = valid & (ty <= y1 // 4) & (tx <= x1 // 8)
                out.append((lbase + qi * hb * wb + ty * wb + tx)[m])
    lines = torch.cat(out)
    return lines


def timed(fn, n, flush):
    evs = []
    for _ in range(n):
        flush()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        evs.append((a, b))
    torch.cuda.synchronize()
    return statistics.median(a.elapsed_time(b) for a, b in evs) * 1e3


def main():
    b, h, w = 8, 55, 128
    dev = torch.device("cuda", 0)
    f1, f2 = synthetic.synthetic_fmaps(b, 256, h, w, stream=3)
    coords = (coords_grid(b, h, w) + torch.from_numpy(synthetic.hash_normal(4, (b, 2, h, w), 4.0))).to(dev)
    tp = _native.corr_pyramid_tiled(f1.to(dev), f2.to(dev), 4)
    lines = window_lines(tp, coords)
    shuffled = lines[torch.randperm(lines.numel(), device=dev)]
    sorted_lines = torch.sort(lines).values
    nb = lookup_bytes(b, tp.dims)
    scratch = torch.ones(1 << 28, device=dev)
    flush = lambda: scratch.sum()  # noqa: E731
    sink = torch.empty(1 << 22, device=dev)
    st = VP(torch.cuda.current_stream().cuda_stream)
    out_bytes = b * h * w * 324 * 4
    outbuf = torch.empty(out_bytes // 4, device=dev)
    rows = torch.empty((b * h * w, 324), device=dev)
    res = {"lines": int(lines.numel()), "line_bytes": int(lines.numel()) * 128, "out_bytes": out_bytes, "algorithmic": nb}
    for blocks in (2048, 8192):
        for name, L in (("query_order", lines), ("shuffled", shuffled), ("sorted", sorted_lines)):
            t = timed(lambda: lib.exp_line_gather(VP(tp.levels[0].data_ptr()), VP(L.data_ptr()), ctypes.c_longlong(L.numel()), VP(sink.data_ptr()), blocks, st), 15, flush)
            res[f"gather_{name}_{blocks}_us"] = round(t, 2)
            res[f"gather_{name}_{blocks}_TBs"] = round(L.numel() * 128 / t / 1e6, 3)
        t = timed(lambda: lib.exp_write_stream(VP(outbuf.data_ptr()), ctypes.c_longlong(out_bytes // 16), blocks, st), 15, flush)
        res[f"write_{blocks}_us"] = round(t, 2)
        res[f"write_{blocks}_TBs"] = round(out_bytes / t / 1e6, 3)
    for blocks in (1024, 2048, 4096):
        for name, L in (("query_order", lines), ("sorted", sorted_lines)):
            t = timed(lambda: lib.exp_line_gather16(VP(tp.levels[0].data_ptr()), VP(L.data_ptr()), ctypes.c_longlong(L.numel()), VP(sink.data_ptr()), blocks, st), 15, flush)
            res[f"gather16_{name}_{blocks}_us"] = round(t, 2)
            res[f"gather16_{name}_{blocks}_TBs"] = round(L.numel() * 128 / t / 1e6, 3)
        nbytes = int(lines.numel()) * 128
        t = timed(lambda: lib.exp_read_stream(VP(tp.levels[0].data_ptr()), ctypes.c_longlong(nbytes // 16), VP(sink.data_ptr()), blocks, st), 15, flush)
        res[f"read_stream_{blocks}_us"] = round(t, 2)
        res[f"read_stream_{blocks}_TBs"] = round(nbytes / t / 1e6, 3)
    t = timed(lambda: _native.corr_lookup_tiled_nhwc(tp, coords, 4, rows), 15, flush)
    res["lookup_nhwc_us"] = round(t, 2)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
