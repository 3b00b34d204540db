"""EXPERIMENT driver: S32 lookup, product (level per workgroup) vs query-major variants; hot (same pyramid every
launch: the touched lines can stay in the 256 MiB Infinity Cache) and cold (3 pyramids in rotation, 6.3 GB)."""
import ctypes
import json
import os
import statistics
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
from optical_flow import _native as N  # noqa: E402

lib = ctypes.CDLL(os.path.join(HERE, "liblookup_s32_exp.so"))
VP = ctypes.c_void_p


def timed(fn, n=60):
    fn(0)
    torch.cuda.synchronize()
    rounds = []
    for _ in range(3):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for i in range(n):
            fn(i)
        b.record()
        b.synchronize()
        rounds.append(a.elapsed_time(b) / n)
    return statistics.median(rounds)


def main():
    b, h, w = 8, 55, 128
    dev = torch.device("cuda", 0)
    pyrs = []
    for s in range(3):
        f1, f2 = synthetic.synthetic_fmaps(b, 256, h, w, stream=3 + s)
        pyrs.append(N.corr_pyramid_tiled(f1.to(dev), f2.to(dev), 4))
    coords = (coords_grid(b, h, w) + torch.from_numpy(synthetic.hash_normal(4, (b, 2, h, w), 4.0))).to(dev)
    dims = pyrs[0].dims
    nbytes = lookup_bytes(b, dims)
    hs = (ctypes.c_int * 4)(*[d[0] for d in dims])
    ws = (ctypes.c_int * 4)(*[d[1] for d in dims])
    ptrs = [(VP * 4)(*[t.data_ptr() for t in p.levels]) for p in pyrs]
    st = VP(torch.cuda.current_stream().cuda_stream)
    outs = [N.s32_empty(b, h, w, 11, dev, zero=True) for _ in range(2)]
    ps = N.S32Slice(outs[0]).ps

    def prod(i, pk):
        return lib.oflow_corr_lookup_tiled_s32(ptrs[pk(i)], hs, ws, 4, VP(coords.data_ptr()), b, h, w, 4,
                                               VP(outs[0].data_ptr()), ctypes.c_longlong(ps), st)

    def qm(i, pk, nt=0, o=1):
        return lib.exp_lookup_s32_qmajor(ptrs[pk(i)], hs, ws, VP(coords.data_ptr()), b, h, w, VP(outs[o].data_ptr()),
                                         ctypes.c_longlong(ps), nt, st)

    hot = lambda i: 0  # noqa: E731
    cold = lambda i: i % 3  # noqa: E731
    assert prod(0, hot) == 0 and qm(0, hot) == 0
    torch.cuda.synchronize()
    same = bool(torch.equal(outs[0], outs[1]))
    res = {"bytes": nbytes, "bit_equal": same}
    nchw = torch.empty(b, 324, h, w, device=dev)

    def prod_nchw(i, pk):
        return lib.oflow_corr_lookup_tiled_f32(ptrs[pk(i)], hs, ws, 4, VP(coords.data_ptr()), b, h, w, 4, VP(nchw.data_ptr()), st)

    variants = {"product_nchw": prod_nchw, "product": prod, "qmajor": qm, "qmajor_nt": lambda i, pk: qm(i, pk, 1)}
    for rnd in range(2):
        for name, fn in variants.items():
            for tag, pk in (("hot", hot), ("cold", cold)):
                t = timed(lambda i: fn(i, pk))
                res.setdefault(f"{name}_{tag}_us", []).append(round(t * 1e3, 1))
    for k, v in list(res.items()):
        if k.endswith("_us"):
            res[k.replace("_us", "_GBs")] = round(nbytes / (min(v) * 1e-6) / 1e9)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
