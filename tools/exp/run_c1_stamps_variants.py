"""Per-workgroup clock stamps of the fused lookup + convc1 kernel variants (oflow_exp_set_convc1_variant /
oflow_exp_set_convc1_stamps), Sintel 55x128 grid, 4 and 8 pairs, N(0, 4^2) px flow. For each variant: event time, then
one stamped launch: median cycles between consecutive stamps (the phases), the median workgroup lifetime, and, per
XCD (s_memtime is per XCD; workgroup i runs on XCD i % 8), the spread of workgroup start / end times relative to the
XCD's first start (p10 / p50 / p90, cycles). VARIANTS=1,3 python tools/exp/run_c1_stamps_variants.py"""
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
from model import synthetic  # noqa: E402
from model.utils import coords_grid  # noqa: E402

DEV = torch.device("cuda", 0)
VARIANTS = [int(v) for v in os.environ.get("VARIANTS", "1,3").split(",")]


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


def pct(v, q):
    v = sorted(v)
    return v[min(len(v) - 1, int(q * len(v)))]


def main():
    lib = N.load()
    lib.oflow_exp_set_convc1_stamps.argtypes = [ctypes.c_void_p]
    lib.oflow_exp_set_convc1_variant.argtypes = [ctypes.c_int]
    h, w = 55, 128
    conv = torch.nn.Conv2d(324, 256, 1).to(DEV)
    cwL = N.convc1_level_weights(conv, 4, 4)
    with torch.inference_mode():
        for b in (4, 8):
            pyrs = []
            for k in range(3):
                f1, f2 = synthetic.synthetic_fmaps(b, 256, h, w, stream=k)
                pyrs.append(N.corr_pyramid_tiled(f1.to(DEV), f2.to(DEV), 4))
            coords = (coords_grid(b, h, w) + torch.from_numpy(synthetic.hash_normal(9, (b, 2, h, w), 4.0))).to(DEV).contiguous()
            y = N.s32_empty(b, h, w, 8, DEV)
            it = [0]

            def fused():
                it[0] = (it[0] + 1) % 3
                N.corr_lookup_convc1(pyrs[it[0]], coords, 4, cwL, N.S32Slice(y))

            for v in VARIANTS:
                lib.oflow_exp_set_convc1_variant(v)
                for _ in range(3):
                    fused()
                torch.cuda.synchronize()
                us = round(min(timeit(fused) for _ in range(3)), 2)
                nwg = (b * h * w + 63) // 64
                st = torch.zeros(nwg * 16, dtype=torch.int64, device=DEV)
                lib.oflow_exp_set_convc1_stamps(st.data_ptr())
                fused()
                torch.cuda.synchronize()
                lib.oflow_exp_set_convc1_stamps(None)
                t = st.view(nwg, 16).cpu().long()
                ns = int((t[0] != 0).sum())
                phases = [round(float((t[:, i + 1] - t[:, i]).double().median())) for i in range(ns - 1)]
                life = [int(t[i, ns - 1] - t[i, 0]) for i in range(nwg)]
                starts, ends = [], []
                for x in range(8):
                    rows = list(range(x, nwg, 8))
                    t0 = min(int(t[i, 0]) for i in rows)
                    starts += [int(t[i, 0]) - t0 for i in rows]
                    ends += [int(t[i, ns - 1]) - t0 for i in rows]
                out = {"variant": v, "pairs": b, "us": us, "stamps": ns, "phase_cycles": phases,
                       "wg_life_p50": pct(life, 0.5), "wg_life_p90": pct(life, 0.9),
                       "start_p10_p50_p90": [pct(starts, q) for q in (0.1, 0.5, 0.9)],
                       "end_p10_p50_p90": [pct(ends, q) for q in (0.1, 0.5, 0.9)], "end_max": max(ends)}
                print(json.dumps(out), flush=True)
            lib.oflow_exp_set_convc1_variant(3)


if __name__ == "__main__":
    main()
