"""Ablation timing of encoder convolutions alone (8 Sintel images 440x1024; needs the -DOFLOW_ABLATE library build, whose
oflow_exp_set_conv_flags bits drop kernel parts: 2 MFMAs, 4 A-operand staging writes, 8 instance-norm partials,
16 output stores). Layers: fnet stem (image in, raw fp32 + partials), cnet stem (image in, folded BN, S32 out), fnet
layer1 conv (normalise-on-load in, raw + partials), cnet layer1 conv (S32 in / out). Prints one JSON line per layer."""
import ctypes
import json
import os
import statistics
import sys

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
for p in (REPO, os.path.join(REPO, "torch-optical-flow_amd"), os.path.join(REPO, "torch-optical-flow_amd", "methods", "raft")):
    sys.path.insert(0, p)

import torch  # noqa: E402

from optical_flow import _native as N  # noqa: E402
from model import RAFT, synthetic  # noqa: E402
from model.extractor import SplitEncoder  # noqa: E402

FLAGS = [0, 2, 4, 8, 16, 2 | 4, 8 | 16, 2 | 4 | 8 | 16]


def timed(fn, n=10, reps=5):
    ts = []
    for _ in range(reps):
        torch.cuda.synchronize()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(n):
            fn()
        b.record()
        b.synchronize()
        ts.append(a.elapsed_time(b) * 1e3 / n)
    return round(statistics.median(ts), 1)


def main():
    dev = torch.device("cuda", 0)
    lib = N.load()
    lib.oflow_exp_set_conv_flags.argtypes = [ctypes.c_int]
    model = RAFT().eval()
    model.load_state_dict(synthetic.synthetic_state_dict(model.state_dict()))
    model = model.to(dev)
    img0, _ = synthetic.synthetic_pair(8, 440, 1024, seed=0)
    x = (2 * (img0.to(dev) / 255.0) - 1.0).contiguous()
    fe, ce = SplitEncoder(model.fnet), SplitEncoder(model.cnet)
    b, h, w = 8, 220, 512
    V = N.S32Slice
    with torch.inference_mode():
        tiles = N.conv_tiles(h, w)
        raw = torch.empty((b * h * w, 64), device=dev)
        part = torch.empty((b, tiles, 64, 3), device=dev)
        s32o = N.s32_empty(b, h, w, 2, dev)
        layers = {
            "fnet stem": lambda: N.conv_s32(N.ImgIn(x), fe.w["stem"], 64, nhwc=raw, stats=part),
            "cnet stem": lambda: N.conv_s32(N.ImgIn(x), ce.w["stem"], 64, act="relu", y0=V(s32o)),
        }
        layers["fnet stem"]()
        alpha, beta = N.norm_stats(part, b, tiles, 64, 64, 1e-5)
        raw2 = torch.empty_like(raw)
        part2 = torch.empty_like(part)
        nin = N.NhwcNormIn(raw, b, h, w, alpha, beta)
        layers["fnet l1 conv"] = lambda: N.conv_s32(nin, fe.w["0.0.conv1"], 64, nhwc=raw2, stats=part2)
        layers["cnet stem"]()
        s32o2 = N.s32_empty(b, h, w, 2, dev)
        layers["cnet l1 conv"] = lambda: N.conv_s32(V(s32o), ce.w["0.0.conv1"], 64, act="relu", y0=V(s32o2))
        for name, fn in layers.items():
            res = {}
            for f in FLAGS:
                lib.oflow_exp_set_conv_flags(f)
                fn()
                res[str(f)] = timed(fn)
            lib.oflow_exp_set_conv_flags(0)
            print(json.dumps({"layer": name, "us_by_flags": res}), flush=True)


if __name__ == "__main__":
    main()
