import os, sys, torch
REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
for p in (REPO, os.path.join(REPO, "torch-optical-flow_amd"), os.path.join(REPO, "torch-optical-flow_amd", "methods", "raft"), os.path.join(REPO, "tests")):
    sys.path.insert(0, p)
from optical_flow import _native as N
import test_gpu_corr_convc1 as T
dev = torch.device("cuda", 0)
for (b, h, w) in [(2, 47, 156), (1, 47, 156), (2, 55, 128)]:
    pyr, coords, conv = T._case(b, h, w, 4, 4, 3.0, seed=7)
    cw = N.convc1_level_weights(conv, 4, 4)
    ref, bound, _ = T._reference(pyr, coords, conv, 4)
    for (b0, b1) in [(0, b), (b - 1, b)]:
        out = N.s32_empty(b1 - b0, h, w, 8, dev, zero=True)
        N.corr_lookup_convc1(pyr.batch_slice(b0, b1), coords[b0:b1], 4, cw, N.S32Slice(out))
        torch.cuda.synchronize()
        got = N.s32_to_f32(out, 256).permute(0, 2, 3, 1).reshape(-1, 256).double()
        r = ref.view(b, h * w, 256)[b0:b1].reshape(-1, 256)
        bad = ~torch.isfinite(got)
        err = (got - r).abs()
        print(b, h, w, (b0, b1), "nonfinite", int(bad.sum()), "maxerr", float(err[~bad].max()) if (~bad).any() else None,
              "bad pixels", torch.nonzero(bad.any(1))[:5].flatten().tolist())
