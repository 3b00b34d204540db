"""In-process A/B of the fused lookup + convc1 kernel (variant 1: the product, liboflow_hip.so) and its experiment
variants (2-5: tools/exp/corr_convc1_variants.hip -> build/exp/libc1var.so, tools/exp/build_c1var.sh): same inputs (Sintel 55x128 grid, N(0, 4^2) px flow, three pyramids in rotation,
cold), 8 pairs (one launch) and 4 pairs (one pair lane); interleaved rounds. Reports whether the outputs are bit-identical
and the largest difference of the S32 values (hi + lo) otherwise.
    python tools/exp/run_c1_variant_ab.py"""
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
VARIANTS = [int(v) for v in os.environ.get("VARIANTS", "1,2,3,4,5,6").split(",")]


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


def s32_values(y):
    """[P, groups * 64] fp16 (S32 lines: hi[32] | lo[32] per group) -> fp32 hi + lo values [P, groups * 32]."""
    v = y.reshape(y.shape[0], -1, 2, 32).float()
    return (v[:, :, 0] + v[:, :, 1]).reshape(y.shape[0], -1)


def check_shape(cw, b, h, w):
    """bit-identity of every variant with variant 1 on one more grid (e.g. KITTI's 47x156: levels 39 and 19 px wide,
    whose right-edge chunk columns cross the level's edge)"""
    f1, f2 = synthetic.synthetic_fmaps(b, 256, h, w, stream=5)
    pyr = N.corr_pyramid_tiled(f1.to(DEV), f2.to(DEV), 4)
    coords = (coords_grid(b, h, w) + torch.from_numpy(synthetic.hash_normal(11, (b, 2, h, w), 6.0))).to(DEV).contiguous()
    vcall = variant_caller(N, cw, coords, b, h, w)
    ys = {}
    with torch.inference_mode():
        for v in VARIANTS:
            ys[v] = N.s32_empty(b, h, w, 8, DEV)
            ys[v].fill_(0)
            vcall(v, pyr, ys[v])
        torch.cuda.synchronize()
    return {f"v{v}": bool(torch.equal(ys[v], ys[VARIANTS[0]])) for v in VARIANTS[1:]}


def main():
    h, w = 55, 128
    conv = torch.nn.Conv2d(324, 256, 1).to(DEV)
    with torch.no_grad():
        conv.weight.mul_(4.0)
    cw = N.convc1_level_weights(conv, 4, 4)
    out = {"kitti47x156_bit_identical": check_shape(cw, 2, 47, 156)}
    for b in (8, 4):
        pyrs = []
        for k in range(3):
            f1, f2 = synthetic.synthetic_fmaps(b, 256, h, w, stream=k)
            pyrs.append(N.corr_pyramid_tiled(f1.to(DEV), f2.to(DEV), 4))
        coords = (coords_grid(b, h, w) + torch.from_numpy(synthetic.hash_normal(9, (b, 2, h, w), 4.0))).to(DEV).contiguous()
        ys = {v: N.s32_empty(b, h, w, 8, DEV) for v in VARIANTS}
        it = [0]
        vcall = variant_caller(N, cw, coords, b, h, w)

        def call(v, pyr):
            vcall(v, pyr, ys[v])

        def arm(v):
            def f():
                it[0] = (it[0] + 1) % 3
                call(v, pyrs[it[0]])
            return f

        same, maxd = True, 0.0
        with torch.inference_mode():
            for k in range(3):
                for v in VARIANTS:
                    ys[v].fill_(0)
                    call(v, pyrs[k])
                torch.cuda.synchronize()
                ref = ys[VARIANTS[0]]
                for v in VARIANTS[1:]:
                    if not torch.equal(ys[v], ref):
                        same = False
                        a, c = s32_values(ys[v].reshape(-1, 8 * 64)), s32_values(ref.reshape(-1, 8 * 64))
                        maxd = max(maxd, float(((a - c).abs() / (c.abs().amax() + 1e-30)).max()))
            res = {}
            for _ in range(4):
                for v in VARIANTS:
                    res.setdefault(v, []).append(timeit(arm(v)))
        out[f"pairs{b}"] = {f"v{k}": {"min": round(min(x), 2), "median": round(statistics.median(x), 2)} for k, x in res.items()}
        out[f"pairs{b}"]["bit_identical"] = same
        out[f"pairs{b}"]["max_rel_diff_of_max"] = maxd
    print(json.dumps({"us": out}))


if __name__ == "__main__":
    main()
