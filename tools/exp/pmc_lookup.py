"""EXPERIMENT: launch each lookup variant 5 times cold (1 GiB read between launches) for rocprofv3 --pmc passes."""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import run_lookup_ab as A  # noqa: E402
import torch  # noqa: E402

from model import synthetic  # noqa: E402
from model.utils import coords_grid  # noqa: E402
from optical_flow import _native  # noqa: E402

VP, I = A.VP, A.I
dev = torch.device("cuda", 0)
b, h, w = 8, 55, 128
f1, f2 = synthetic.synthetic_fmaps(b, 256, h, w, stream=3)
coords = (coords_grid(b, h, w) + torch.from_numpy(synthetic.hash_normal(4, (b, 2, h, w), 4.0))).to(dev)
tp = _native.corr_pyramid_tiled(f1.to(dev), f2.to(dev), 4)
dims = tp.dims
ptrs = (VP * 4)(*[t.data_ptr() for t in tp.levels])
hs = (I * 4)(*[d[0] for d in dims])
ws = (I * 4)(*[d[1] for d in dims])
st = VP(torch.cuda.current_stream().cuda_stream)
rows352 = torch.empty((b * h * w, 352), device=dev)
rows324 = torch.empty((b * h * w, 324), device=dev)
scratch = torch.ones(1 << 28, device=dev)
for _ in range(5):
    scratch.sum()
    A.lib.r01_corr_lookup_tiled_nhwc_f32(ptrs, hs, ws, 4, VP(coords.data_ptr()), b, h, w, 4, VP(rows352.data_ptr()), 352, st)
    scratch.sum()
    _native.corr_lookup_tiled_nhwc(tp, coords, 4, rows324)
    scratch.sum()
    _native.corr_lookup_tiled(tp, coords, 4)
torch.cuda.synchronize()
print("done")
