"""Debug: the z|r GRU epilogue test repeated, max errors and where (OFLOW_LIB / OFLOW_OPS_LIB pick the build)."""
import os, sys
REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(REPO, "torch-optical-flow_amd"))
import torch
import torch.nn.functional as F
from optical_flow import _native as N
DEV = torch.device("cuda", 0)
for rep in range(4):
    g = torch.Generator().manual_seed(11)
    b, h, w, ch = 2, 8, 36, 128
    hx = torch.randn(b, 384, h, w, generator=g).to(DEV)
    hx[:, :ch] = torch.tanh(hx[:, :ch])
    hmaster = hx[:, :ch].permute(0, 2, 3, 1).reshape(-1, ch).contiguous()
    hx_s = N.s32_from_f32(hx)
    rhx_s = hx_s.clone()
    wz, wr, wq = ((torch.randn(ch, 384, 1, 5, generator=g) * 0.02).to(DEV) for _ in range(3))
    bz, br, bq = (torch.randn(ch, generator=g).to(DEV) for _ in range(3))
    czr = N.ConvWeights(torch.cat([wz, wr]), torch.cat([bz, br]), 256)
    z = torch.empty(b * h * w, ch, device=DEV)
    N.conv_s32(N.S32Slice(hx_s), czr, 128, epilogue=1, y0=N.S32Slice(rhx_s, 0, 4), gru_h=hmaster, gru_z=z)
    hxr = N.s32_to_f32(hx_s).double()
    zr_ref = torch.sigmoid(F.conv2d(hxr, wz.double(), bz.double(), padding=(0, 2)))
    r_ref = torch.sigmoid(F.conv2d(hxr, wr.double(), br.double(), padding=(0, 2)))
    zg = z.view(b, h, w, ch).permute(0, 3, 1, 2).double()
    rh_ref = r_ref * hx[:, :ch].double()
    rhx = N.s32_to_f32(rhx_s).double()
    e = (rhx[:, :ch] - rh_ref).abs()
    bad = (e > 2e-6).nonzero()
    print(rep, "z", float((zg - zr_ref).abs().max()), "rh", float(e.max()), "nbad", len(bad), bad[:6].tolist(), flush=True)
    if len(bad):
        i = bad[0].tolist()
        print("   got", float(rhx[i[0], i[1], i[2], i[3]]), "ref", float(rh_ref[i[0], i[1], i[2], i[3]]),
              "h", float(hx[i[0], i[1], i[2], i[3]]), "hs", float(hxr[i[0], i[1], i[2], i[3]]), flush=True)
