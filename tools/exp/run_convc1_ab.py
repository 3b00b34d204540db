"""In-process A/B: the lookup fused into convc1 (oflow_corr_lookup_convc1_s32) vs the unfused pair (NHWC lookup rows ->
oflow_conv_s32 OFLOW_IN_F32), Sintel 55x128 grid, 8 pairs (one launch) and 4 pairs (one pair lane), N(0, 4^2) px
flow; three pyramids in rotation so nothing survives in the 256 MiB Infinity Cache ("cold"). Prints one JSON line."""
import json
import math
import os
import statistics
import sys

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
for p in (REPO, os.path.join(REPO, "torch-optical-flow_amd"), os.path.join(REPO, "torch-optical-flow_amd", "methods", "raft")):
    sys.path.insert(0, p)

import torch  # noqa: E402

from optical_flow import _native as N  # noqa: E402
from model import synthetic  # noqa: E402
from model.utils import coords_grid  # noqa: E402

DEV = torch.device("cuda", 0)


def timeit(fn, reps=20):
    ts = []
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        torch.cuda.synchronize()
        ts.append(a.elapsed_time(b) * 1e3)
    return statistics.median(ts)


def main():
    h, w = 55, 128
    out = {}
    conv = torch.nn.Conv2d(324, 256, 1).to(DEV)
    with torch.no_grad():
        conv.weight.mul_(4.0)
    cwL = N.convc1_level_weights(conv, 4, 4)
    cw = N.ConvWeights(conv.weight, conv.bias, 256)
    for b in (8, 4):
        pyrs = []
        for k in range(3):
            f1, f2 = synthetic.synthetic_fmaps(b, 256, h, w, stream=k)
            pyrs.append(N.corr_pyramid_tiled(f1.to(DEV), f2.to(DEV), 4))
        coords = (coords_grid(b, h, w) + torch.from_numpy(synthetic.hash_normal(9, (b, 2, h, w), 4.0))).to(DEV).contiguous()
        y = N.s32_empty(b, h, w, 8, DEV)
        rows = torch.empty((b * h * w, 324), device=DEV)
        it = [0]

        def nxt():
            it[0] = (it[0] + 1) % 3
            return pyrs[it[0]]

        def fused():
            N.corr_lookup_convc1(nxt(), coords, 4, cwL, N.S32Slice(y))

        def lookup():
            N.corr_lookup_tiled_nhwc(nxt(), coords, 4, rows)

        def c1():
            N.conv_s32(N.F32In(rows, b, h, w), cw, 128, "relu", y0=N.S32Slice(y))

        def unfused():
            lookup()
            c1()

        with torch.inference_mode():
            for f in (fused, unfused):
                for _ in range(3):
                    f()
            torch.cuda.synchronize()
            res = {}
            for rnd in range(3):  # interleaved rounds
                for name, f in (("fused", fused), ("lookup", lookup), ("convc1", c1), ("unfused", unfused)):
                    res.setdefault(name, []).append(timeit(f))
        out[f"pairs{b}"] = {k: round(min(v), 2) for k, v in res.items()}
        q = b * h * w
        flops = q * 12 * 32 * 256 * 6
        out[f"pairs{b}"]["fused_tflops_f16_executed"] = round(flops / (out[f"pairs{b}"]["fused"] * 1e-6) / 1e12, 1)
    print(json.dumps({"us": out}))


if __name__ == "__main__":
    main()
