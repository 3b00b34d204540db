import os, sys
REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
PKG = os.path.join(REPO, "torch-optical-flow_amd")
for p in (REPO, PKG, os.path.join(PKG, "methods", "raft")):
    sys.path.insert(0, p)
import torch
from model import synthetic
from model.utils import coords_grid
from optical_flow import _native as N
torch.set_printoptions(precision=3, linewidth=200, sci_mode=False)
dev = torch.device("cuda", 0)
b, h, w, r = 1, 16, 16, 2
f1, f2 = synthetic.synthetic_fmaps(b, 64, h, w, stream=63)
f1, f2 = f1.to(dev), f2.to(dev)
coords = coords_grid(b, h, w).to(dev)
tp = N.corr_pyramid_tiled(f1, f2, 4)
cp = N.corr_pyramid(f1, f2, 4)
a = N.corr_lookup_tiled(tp, coords, r)
c = N.corr_lookup(cp, coords, r)
torch.cuda.synchronize()
for (y, x) in [(0, 0), (2, 0), (5, 7)]:
    print("query", y, x)
    print(" got  L0:", a[0, :25, y, x].view(5, 5).t())
    print(" want L0:", c[0, :25, y, x].view(5, 5).t())
    q = y * w + x
    P = cp[0][q, 0]
    print(" pyr window:", P[max(0,y-2):y+3, max(0,x-2):x+3])
