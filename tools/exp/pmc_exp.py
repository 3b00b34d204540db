"""EXPERIMENT: run each lookup variant a few times (for rocprofv3 --pmc) on Sintel x8."""
import ctypes, os, sys
HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import run_lookup_exp as R
import torch
from model import synthetic
from model.utils import coords_grid
from optical_flow import _native
VP = ctypes.c_void_p
dev = torch.device("cuda", 0)
b, h, w = 8, 55, 128
f1, f2 = synthetic.synthetic_fmaps(b, 256, h, w, stream=3)
pyr = _native.corr_pyramid(f1.to(dev), f2.to(dev), 4)
coords = (coords_grid(b, h, w) + torch.from_numpy(synthetic.hash_normal(4, (b, 2, h, w), 4.0))).to(dev)
ref = _native.corr_lookup(pyr, coords, 4)
dims = [(int(p.shape[2]), int(p.shape[3])) for p in pyr]
st = VP(torch.cuda.current_stream().cuda_stream)
lvp = (VP * 4)(*[p.data_ptr() for p in pyr]); hs = (ctypes.c_int * 4)(*[d[0] for d in dims]); ws = (ctypes.c_int * 4)(*[d[1] for d in dims])
out = torch.empty_like(ref)
for mode in (0, 3, 4):
    for _ in range(3):
        assert R.lib.exp_lookup_ablate(lvp, hs, ws, mode, 64, VP(coords.data_ptr()), b, h * w, VP(out.data_ptr()), st) == 0
q = b * h * w
for bh, bw, qpb in [(4, 4, 32), (4, 8, 16), (1, 32, 16)]:
    blk = []
    for p, (hl, wl) in zip(pyr, dims):
        o = torch.empty(q * (-(-hl // bh)) * (-(-wl // bw)) * bh * bw, device=dev)
        R.lib.exp_relayout(VP(p.data_ptr()), VP(o.data_ptr()), ctypes.c_longlong(q), hl, wl, bh, bw, st)
        blk.append(o)
    ptrs = (VP * 4)(*[x.data_ptr() for x in blk])
    for _ in range(3):
        assert R.lib.exp_lookup_blocked(ptrs, hs, ws, bh, bw, 1000 + qpb, VP(coords.data_ptr()), b, h * w, VP(out.data_ptr()), st) == 0
torch.cuda.synchronize()
print("done")
