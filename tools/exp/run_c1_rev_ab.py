"""In-process A/B of the fused lookup + convc1 kernel between this tree's liboflow_hip.so and another build (OLD_LIB,
e.g. tools/build_rev.sh HEAD base): same inputs (Sintel 55x128 grid, N(0, 4^2) px flow, three pyramids in rotation,
cold), 8 pairs (one launch) and 4 pairs (one pair lane); interleaved rounds; outputs compared bit for bit.
    OLD_LIB=build/rev_base/_lib/liboflow_hip.so python tools/exp/run_c1_rev_ab.py"""
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
    new = N.load()
    old = ctypes.CDLL(os.environ["OLD_LIB"])
    old.oflow_corr_lookup_convc1_s32.restype = ctypes.c_int
    old.oflow_corr_lookup_convc1_s32.argtypes = new.oflow_corr_lookup_convc1_s32.argtypes
    h, w = 55, 128
    conv = torch.nn.Conv2d(324, 256, 1).to(DEV)
    with torch.no_grad():
        conv.weight.mul_(4.0)
    cw = N.convc1_level_weights(conv, 4, 4)
    out = {}
    for b in (8, 4):
        pyrs = []
        for k in range(3):
            f1, f2 = synthetic.synthetic_fmaps(b, 256, h, w, stream=k)
            pyrs.append(N.corr_pyramid_tiled(f1.to(DEV), f2.to(DEV), 4))
        coords = (coords_grid(b, h, w) + torch.from_numpy(synthetic.hash_normal(9, (b, 2, h, w), 4.0))).to(DEV).contiguous()
        ys = {"new": N.s32_empty(b, h, w, 8, DEV), "old": N.s32_empty(b, h, w, 8, DEV)}
        it = [0]

        def call(lib, y, pyr):
            ptrs = (ctypes.c_void_p * N.MAX_LEVELS)(*[t.data_ptr() for t in pyr.levels])
            hs = (ctypes.c_int * N.MAX_LEVELS)(*[d[0] for d in pyr.dims])
            ws = (ctypes.c_int * N.MAX_LEVELS)(*[d[1] for d in pyr.dims])
            st = lib.oflow_corr_lookup_convc1_s32(ptrs, hs, ws, 4, coords.data_ptr(), b, h, w, 4, cw.pack.data_ptr(),
                                                   cw.wscale.data_ptr(), cw.bias.data_ptr(), y.data_ptr(), 8 * 128,
                                                   ctypes.c_void_p(torch.cuda.current_stream().cuda_stream))
            assert st == 0, st

        def arm(name, lib):
            def f():
                it[0] = (it[0] + 1) % 3
                call(lib, ys[name], pyrs[it[0]])
            return f

        arms = {"new": arm("new", new), "old": arm("old", old)}
        with torch.inference_mode():
            for k in range(3):
                call(new, ys["new"], pyrs[k])
                call(old, ys["old"], pyrs[k])
                torch.cuda.synchronize()
                assert torch.equal(ys["new"], ys["old"]), f"outputs differ (pyramid {k})"
            res = {}
            for _ in range(4):
                for name, f in arms.items():
                    res.setdefault(name, []).append(timeit(f))
        out[f"pairs{b}"] = {k: {"min": round(min(v), 2), "median": round(statistics.median(v), 2)} for k, v in res.items()}
    print(json.dumps({"us": out, "bit_identical": True}))


if __name__ == "__main__":
    main()
