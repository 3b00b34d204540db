"""Times the inference-I/O kernels (csrc/flow_io.hip) on the GPU: flow2rgb (stats + colour pass) and flow_pack on
Sintel-size flow fields, against their HBM-byte rooflines. Prints one JSON line per kernel.
usage: python tools/iobench.py [--batch 8] [--reps 50]"""
import argparse
import json
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "torch-optical-flow_amd")]
import optical_flow  # noqa: E402
from optical_flow import _native  # noqa: E402


def timed(fn, reps):
    for _ in range(3):
        fn()
    s = torch.cuda.current_stream()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    for _ in range(reps):
        fn()
    e1.record(s)
    e1.synchronize()
    return e0.elapsed_time(e1) / reps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=8)
    ap.add_argument("--reps", type=int, default=50)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    b, h, w = a.batch, 436, 1024
    flow = torch.randn(b, 2, h, w, device=dev) * 10
    px = b * h * w
    for method in ("baker", "hsv", "meister"):
        ms = timed(lambda: optical_flow.flow2rgb(flow, method), a.reps)
        byts = px * (8 + 8 + 12)  # stats read + colour pass read + write
        print(json.dumps({"kernel": f"flow2rgb_{method}", "shape": [b, 2, h, w], "ms": round(ms, 4),
                          "algorithmic_bytes": byts, "GB/s": round(byts / ms / 1e6, 1),
                          "frac_hbm": round(byts / ms / 1e6 / 8000, 3)}))
    ms = timed(lambda: _native.flow_pack(flow, 2, False), a.reps)
    print(json.dumps({"kernel": "flow_pack_flo", "shape": [b, 2, h, w], "ms": round(ms, 4), "algorithmic_bytes": px * 16,
                      "GB/s": round(px * 16 / ms / 1e6, 1), "frac_hbm": round(px * 16 / ms / 1e6 / 8000, 3)}))


if __name__ == "__main__":
    main()
