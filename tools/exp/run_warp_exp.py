"""EXPERIMENT driver: direct-gather vs LDS-staged bilinear warp on (8, 3, 436, 1024) frames: the SURVEY workload
(i.i.d. N(0, 8^2) px flow), a smooth flow (+-20 px, low frequency) and zero flow; interleaved rounds, one process."""
import ctypes
import json
import math
import os
import statistics
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
PKG = os.path.join(REPO, "torch-optical-flow_amd")
for p in (REPO, PKG, os.path.join(PKG, "methods", "raft")):
    sys.path.insert(0, p)

import torch  # noqa: E402

import optical_flow  # noqa: E402
from model import synthetic  # noqa: E402

lib = ctypes.CDLL(os.path.join(HERE, "libwarp_exp.so"))
VP = ctypes.c_void_p


def timed(fn, n=50):
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
    dev = torch.device("cuda", 0)
    B, C, H, W = 8, 3, 436, 1024
    frame, _ = synthetic.synthetic_pair(B, H, W, seed=1)
    frame = frame.to(dev)
    yy, xx = torch.meshgrid(torch.arange(H, dtype=torch.float32), torch.arange(W, dtype=torch.float32), indexing="ij")
    smooth = torch.stack([20 * torch.sin(xx / 97.0 + yy / 61.0), 20 * torch.cos(xx / 83.0 - yy / 71.0)])
    flows = {
        "iid_sigma8": torch.from_numpy(synthetic.hash_normal(5, (B, 2, H, W), 8.0)),
        "smooth_20px": smooth.expand(B, 2, H, W).contiguous(),
        "zero": torch.zeros(B, 2, H, W),
        "iid_sigma2": torch.from_numpy(synthetic.hash_normal(6, (B, 2, H, W), 2.0)),
        "iid_sigma4": torch.from_numpy(synthetic.hash_normal(7, (B, 2, H, W), 4.0)),
    }
    nbytes = (2 * C + 2) * 4 * B * H * W
    st = VP(torch.cuda.current_stream().cuda_stream)
    out = {}
    for name, px in flows.items():
        fl = optical_flow.normalize(px).to(dev)
        o = [torch.empty_like(frame) for _ in range(2)]
        for w in (0, 1):
            lib.exp_warp(w, VP(frame.data_ptr()), VP(fl.data_ptr()), B, C, H, W, VP(o[w].data_ptr()), st)
        torch.cuda.synchronize()
        res = {"bit_equal": bool(torch.equal(o[0], o[1]))}
        ts = {0: [], 1: []}
        for _ in range(5):
            for w in (0, 1):
                ts[w].append(timed(lambda: lib.exp_warp(w, VP(frame.data_ptr()), VP(fl.data_ptr()), B, C, H, W, VP(o[w].data_ptr()), st)))
        for w, tag in ((0, "direct"), (1, "staged")):
            t = statistics.median(ts[w])
            res[tag + "_us"] = round(t * 1e3, 1)
            res[tag + "_GBs"] = round(nbytes / (t * 1e-3) / 1e9)
        out[name] = res
        print(name, res, flush=True)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
