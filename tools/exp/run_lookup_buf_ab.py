"""In-process A/B of the tiled CorrBlock lookup's gathers (oflow_exp_set_lookup_buf: 0 = exec-masked scalar loads,
1 = unconditional buffer loads with out-of-level sentinels) at the bench workload's shape (8 Sintel pairs, 55 x 128,
4 levels, radius 4): two pyramids alternating (cold, as bench.py's corr_lookup_api leg) and one (hot); NCHW and NHWC
outputs compared bit for bit across the settings. Prints one JSON line. (Run on the r06 s16 tree; the BUF gathers were
then made the default and the hook removed: profiles/r06/r6s16_lookup_ab.log.)"""
import ctypes
import json
import os
import statistics
import sys

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
for p in (REPO, os.path.join(REPO, "torch-optical-flow_amd"), os.path.join(REPO, "torch-optical-flow_amd", "methods", "raft")):
    sys.path.insert(0, p)

import torch  # noqa: E402

from bench import lookup_bytes  # noqa: E402
from model import synthetic  # noqa: E402
from model.utils import coords_grid  # noqa: E402
from optical_flow import _native  # noqa: E402


def main():
    lib = _native.load()
    hook = lib.oflow_exp_set_lookup_buf
    hook.argtypes, hook.restype = [ctypes.c_int], None
    b, h, w = 8, 55, 128
    dev = torch.device("cuda", 0)
    pyrs, coords = [], []
    for k in range(2):
        f1, f2 = synthetic.synthetic_fmaps(b, 256, h, w, stream=3 + k)
        pyrs.append(_native.corr_pyramid_tiled(f1.to(dev), f2.to(dev), 4))
        coords.append((coords_grid(b, h, w) + torch.from_numpy(synthetic.hash_normal(4 + k, (b, 2, h, w), 4.0))).to(dev))
    dims = [(h >> l, w >> l) for l in range(4)]
    nbytes = lookup_bytes(b, dims)
    rows = torch.empty(b * h * w, 324, device=dev)
    outs = {}
    for v in (0, 1):
        hook(v)
        outs[v] = (_native.corr_lookup_tiled(pyrs[0], coords[0], 4).clone(),
                   _native.corr_lookup_tiled_nhwc(pyrs[0], coords[0], 4, rows).clone())
    res = {"algorithmic_bytes": nbytes,
           "bit_identical": bool(torch.equal(outs[0][0], outs[1][0]) and torch.equal(outs[0][1], outs[1][1]))}
    for mode in ("cold", "hot"):
        t = {0: [], 1: []}
        for _ in range(5):
            for v in (0, 1):
                hook(v)
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for i in range(20):
                    k = i % 2 if mode == "cold" else 0
                    _native.corr_lookup_tiled(pyrs[k], coords[k], 4)
                e1.record()
                e1.synchronize()
                t[v].append(e0.elapsed_time(e1) / 20 * 1e3)
        for v in (0, 1):
            us = statistics.median(t[v])
            res[f"{mode}_v{v}_us"] = round(us, 2)
            res[f"{mode}_v{v}_frac"] = round(nbytes / (us * 1e-6) / 8e12, 4)
    hook(0)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
