"""Per-workgroup clock stamps of the fused lookup + convc1 kernel (variant 1, the product) and its experiment variants
(2-5, build/exp/libc1var.so; see run_c1_variant_ab.py), Sintel 55x128 grid, 4 and 8 pairs, N(0, 4^2) px flow. For each variant: event time, then
one stamped launch: median cycles between consecutive stamps (the phases) and the workgroup lifetime (p50 / p90; only
in-workgroup differences: s_memtime is not synchronised across XCDs). VARIANTS=1,3 python tools/exp/run_c1_stamps_variants.py"""
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


def timeit(fn, reps=20, burst=5):
    """median GPU time per launch (us) of `burst` back-to-back launches queued behind a spin kernel, so the host's
    launch overhead (the product wrapper's Python checks vs a bare ctypes call) is not in the events' interval"""
    ts = []
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda._sleep(2_000_000)
        a.record()
        for _ in range(burst):
            fn()
        b.record()
        torch.cuda.synchronize()
        ts.append(a.elapsed_time(b) * 1e3 / burst)
    return statistics.median(ts)


def variant_caller(N, cw, coords, b, h, w):
    """call(v, pyr, y, stamps=None): variant 1 = the product kernel (N.corr_lookup_convc1; stamps through the product's
    hook), variants 2-5 = build/exp/libc1var.so (tools/exp/build_c1var.sh), same arguments."""
    exp = ctypes.CDLL(os.path.join(REPO, "build", "exp", "libc1var.so"))
    exp.oflow_exp_convc1_variant.restype = ctypes.c_int
    P, I = ctypes.c_void_p, ctypes.c_int
    exp.oflow_exp_convc1_variant.argtypes = [I, ctypes.POINTER(ctypes.c_void_p), ctypes.POINTER(I), ctypes.POINTER(I), I, P,
                                             I, I, I, I, P, P, P, P, ctypes.c_longlong, P, P]
    lib = N.load()
    lib.oflow_exp_set_convc1_stamps.argtypes = [ctypes.c_void_p]

    def call(v, pyr, y, stamps=None):
        if v == 1:
            lib.oflow_exp_set_convc1_stamps(stamps)
            N.corr_lookup_convc1(pyr, coords, 4, cw, N.S32Slice(y))
            lib.oflow_exp_set_convc1_stamps(None)
            return
        ptrs = (ctypes.c_void_p * N.MAX_LEVELS)(*[t.data_ptr() for t in pyr.levels])
        hs = (ctypes.c_int * N.MAX_LEVELS)(*[d[0] for d in pyr.dims])
        ws = (ctypes.c_int * N.MAX_LEVELS)(*[d[1] for d in pyr.dims])
        st = exp.oflow_exp_convc1_variant(v, ptrs, hs, ws, 4, coords.data_ptr(), b, h, w, 4, cw.pack.data_ptr(),
                                          cw.wscale.data_ptr(), cw.bias.data_ptr(), y.data_ptr(), 8 * 128, stamps,
                                          ctypes.c_void_p(torch.cuda.current_stream().cuda_stream))
        assert st == 0, st
    return call


def pct(v, q):
    v = sorted(v)
    return v[min(len(v) - 1, int(q * len(v)))]


def main():
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
            vcall = variant_caller(N, cwL, coords, b, h, w)

            for v in VARIANTS:
                def fused(stamps=None):
                    it[0] = (it[0] + 1) % 3
                    vcall(v, pyrs[it[0]], y, stamps)

                for _ in range(3):
                    fused()
                torch.cuda.synchronize()
                us = round(min(timeit(fused) for _ in range(3)), 2)
                nwg = (b * h * w + 63) // 64
                st = torch.zeros(nwg * 16, dtype=torch.int64, device=DEV)
                fused(st.data_ptr())
                torch.cuda.synchronize()
                t = st.view(nwg, 16).cpu().long()
                t = t[t[:, 0] != 0]  # variants with larger workgroups fill fewer rows
                nwg = t.shape[0]
                ns = int((t[0] != 0).sum())
                phases = [round(float((t[:, i + 1] - t[:, i]).double().median())) for i in range(ns - 1)]
                life = [int(t[i, ns - 1] - t[i, 0]) for i in range(nwg)]
                out = {"variant": v, "pairs": b, "us": us, "stamps": ns, "phase_cycles": phases,
                       "wg_life_p50": pct(life, 0.5), "wg_life_p90": pct(life, 0.9)}
                print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
