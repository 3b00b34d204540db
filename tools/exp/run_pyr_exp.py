"""EXPERIMENT: corr_pyramid variants (GEMM-only, k-pair LDS reads) vs the product kernel."""
import ctypes, json, os, statistics, sys
HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
PKG = os.path.join(REPO, "torch-optical-flow_amd")
for p in (REPO, PKG, os.path.join(PKG, "methods", "raft")):
    sys.path.insert(0, p)
import torch
from model import synthetic
from optical_flow import _native
from bench import pyramid_cost
lib = ctypes.CDLL(os.path.join(HERE, "libpyr_exp.so"))
VP = ctypes.c_void_p

def timed(fn, n=50):
    """Mean per-launch time of n back-to-back launches between one event pair (median of 3 rounds): the queue
    stays ahead of the GPU, so host launch latency is not in the number."""
    fn()
    torch.cuda.synchronize()
    rounds = []
    for _ in range(3):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(n):
            fn()
        b.record()
        b.synchronize()
        rounds.append(a.elapsed_time(b) / n)
    return statistics.median(rounds)

for name, (b, h, w) in {"sintel8": (8, 55, 128), "corr4": (4, 128, 128)}.items():
    dev = torch.device("cuda", 0)
    f1, f2 = synthetic.synthetic_fmaps(b, 256, h, w, stream=3)
    f1, f2 = f1.to(dev), f2.to(dev)
    ref = _native.corr_pyramid(f1, f2, 4)
    dims = [(int(p.shape[2]), int(p.shape[3])) for p in ref]
    flops, _ = pyramid_cost(b, dims)
    out = [torch.empty_like(p) for p in ref]
    ptrs = (VP * 4)(*[o.data_ptr() for o in out])
    st = VP(torch.cuda.current_stream().cuda_stream)
    res = {"shape": name}
    t = timed(lambda: _native.corr_pyramid(f1, f2, 4))
    res["product"] = (round(t, 4), round(flops / t / 1e9, 1))
    for ns, b64 in [(0, 0), (1, 0), (0, 1), (1, 1)]:
        go = lambda: lib.exp_pyramid(VP(f1.data_ptr()), VP(f2.data_ptr()), b, 256, h, w, ptrs, ns, b64, st)
        assert go() == 0
        torch.cuda.synchronize()
        err = max(float((o - r).abs().max()) for o, r in zip(out, ref)) if ns == 0 else None
        t = timed(go)
        res[f"ns{ns}_b64{b64}"] = (round(t, 4), round(flops / t / 1e9, 1), err)
    print(json.dumps(res), flush=True)
