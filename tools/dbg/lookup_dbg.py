"""Debug: segment-DMA lookup vs canonical lookup, mismatch locations."""
import os, sys
REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
PKG = os.path.join(REPO, "torch-optical-flow_amd")
for p in (REPO, PKG, os.path.join(PKG, "methods", "raft")):
    sys.path.insert(0, p)
import torch
from model import synthetic
from model.utils import coords_grid
from optical_flow import _native as N
dev = torch.device("cuda", 0)
for (b, h, w, r, sigma) in [(1, 16, 16, 2, 0.0), (2, 47, 156, 2, 0.0), (2, 47, 156, 4, 0.0), (2, 47, 156, 4, 4.0), (8, 55, 128, 4, 4.0)]:
    f1, f2 = synthetic.synthetic_fmaps(b, 64, h, w, stream=63)
    f1, f2 = f1.to(dev), f2.to(dev)
    coords = (coords_grid(b, h, w) + torch.from_numpy(synthetic.hash_normal(64, (b, 2, h, w), sigma))).to(dev)
    tp = N.corr_pyramid_tiled(f1, f2, 4)
    cp = N.corr_pyramid(f1, f2, 4)
    a = N.corr_lookup_tiled(tp, coords, r)
    c = N.corr_lookup(cp, coords, r)
    torch.cuda.synchronize()
    d = (a - c).abs()
    bad = ~(a == c)
    k = 2 * r + 1
    print(f"b{b} {h}x{w} r{r} s{sigma}: mismatches {int(bad.sum())}/{bad.numel()} max {float(d[torch.isfinite(d)].max()) if torch.isfinite(d).any() else 'nan'} nan_a {int(torch.isnan(a).sum())} nan_c {int(torch.isnan(c).sum())}")
    if bad.any():
        idx = bad.nonzero()
        lv = idx[:, 1] // (k * k)
        print("  per level:", [int((lv == l).sum()) for l in range(4)])
        print("  per batch:", [int((idx[:, 0] == i).sum()) for i in range(b)])
        qs = (idx[:, 0] * h * w + idx[:, 2] * w + idx[:, 3])
        print("  queries (first):", sorted(set(qs.tolist()))[:20], " count", len(set(qs.tolist())))
        print("  q mod 16 hist:", torch.bincount(qs % 16, minlength=16).tolist())
        kk = idx[:, 1] % (k * k)
        print("  tap hist:", torch.bincount(kk, minlength=k * k).tolist())
        i0 = idx[0]
        print("  first:", i0.tolist(), float(a[tuple(i0)]), float(c[tuple(i0)]))
    rows = torch.full((b * h * w, 4 * k * k), 7.0, device=dev)
    N.corr_lookup_tiled_nhwc(tp, coords, r, rows)
    torch.cuda.synchronize()
    print("  nhwc==canonical:", bool(torch.equal(rows.view(b, h, w, -1), c.permute(0, 2, 3, 1))), " nhwc==seg nchw:", bool(torch.equal(rows.view(b, h, w, -1), a.permute(0, 2, 3, 1))))
