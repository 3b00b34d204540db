"""On-the-fly fp16 correlation (AlternateCorrBlock; BASELINE configs[4]) against the dense fp32 oracle.

Tolerances: fp16 features (2^-11 relative rounding) with fp32 MFMA accumulation give corr errors of a few 1e-4
(estimate: sqrt(C)*E|f1 f2|*4e-4/sqrt(C) ~ 5e-4 rms at C=256), so lookup outputs are checked at mean |d| <= 1e-3,
max |d| <= 2e-2; end-to-end flow at SURVEY §8(c)'s fp16 bar: mean EPE <= 2e-3 px, max <= 2e-2 px.
"""
import numpy as np
import pytest
import torch

from model import RAFT, AlternateCorrBlock, CorrBlock, InputPadder, synthetic
from model.utils import coords_grid
from optical_flow import _native
from oracle import corr as ocorr

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)


def _check(got, ref, mean_tol=1e-3, max_tol=2e-2):
    d = (got.detach().float().cpu() - ref.detach().float().cpu()).abs()
    assert float(d.mean()) <= mean_tol and float(d.max()) <= max_tol, (float(d.mean()), float(d.max()))


@pytest.mark.parametrize("sigma", [0.0, 3.0, 30.0])
@pytest.mark.parametrize("shape", [(1, 16, 20), (2, 19, 37)])
def test_otf_matches_dense_oracle(shape, sigma):
    b, h, w = shape
    f1, f2 = synthetic.synthetic_fmaps(b, 256, h, w, stream=21)
    coords = ocorr.coords_grid(b, h, w) + torch.from_numpy(synthetic.hash_normal(22, (b, 2, h, w), sigma))
    ref = ocorr.corr_lookup(ocorr.corr_pyramid(f1, f2, 4), coords, 4)
    blk = AlternateCorrBlock(f1.to(DEV), f2.to(DEV))
    got = blk(coords.to(DEV))
    assert got.shape == ref.shape and got.dtype == torch.float32
    _check(got, ref)


def test_otf_radius_and_levels():
    b, h, w = 1, 24, 32
    f1, f2 = synthetic.synthetic_fmaps(b, 64, h, w, stream=23)
    coords = ocorr.coords_grid(b, h, w) + torch.from_numpy(synthetic.hash_normal(24, (b, 2, h, w), 2.0))
    for radius, levels in ((0, 1), (2, 3), (3, 4)):
        ref = ocorr.corr_lookup(ocorr.corr_pyramid(f1, f2, levels), coords, radius)
        got = AlternateCorrBlock(f1.to(DEV), f2.to(DEV), num_levels=levels, radius=radius)(coords.to(DEV))
        _check(got, ref)


def test_otf_feature_pyramid_is_pooled_fmap2():
    f1, f2 = synthetic.synthetic_fmaps(1, 64, 20, 24, stream=25)
    f1h, f2h = _native.otf_prepare(f1.to(DEV), f2.to(DEV), 3)
    assert torch.equal(f1h.cpu(), (f1 * 0.125).permute(0, 2, 3, 1).half())  # 1/sqrt(64) exact
    lvl = f2
    for l in range(3):
        assert torch.equal(f2h[l].cpu(), lvl.permute(0, 2, 3, 1).half()), l
        lvl = torch.nn.functional.avg_pool2d(lvl, 2, stride=2)


def test_otf_matches_dense_kernel_at_1080p():
    """configs[4] shape: 1080x1920 -> 135 x 240 queries, dense fp32 HIP path vs on-the-fly fp16 path."""
    b, h, w = 1, 135, 240
    f1, f2 = synthetic.synthetic_fmaps(b, 256, h, w, stream=26)
    f1, f2 = f1.to(DEV), f2.to(DEV)
    coords = (coords_grid(b, h, w) + torch.from_numpy(synthetic.hash_normal(27, (b, 2, h, w), 6.0))).to(DEV)
    dense = CorrBlock(f1, f2)(coords)
    otf = AlternateCorrBlock(f1, f2)(coords)
    _check(otf, dense)


def test_raft_alternate_corr_matches_reference_flow(golden):
    g = golden("raft_e2e")
    for tag in ("small", "sintel"):
        b, h, w, iters, s, seed = (int(v) for v in g[f"{tag}_cfg"])
        img0, img1 = synthetic.synthetic_pair(b, h, w, seed=seed)
        padder = InputPadder(img0.shape, mode=str(g[f"{tag}_mode"]))
        model = RAFT(alternate_corr=True).eval()
        model.load_state_dict(synthetic.synthetic_state_dict(model.state_dict()))
        model = model.to(DEV)
        with torch.inference_mode():
            low, up = model(*(x.to(DEV) for x in padder.pad(img0, img1)), iters=iters, test_mode=True)
        up = padder.unpad(up)[..., ::s, ::s].cpu()
        e = torch.norm(up - torch.from_numpy(g[f"{tag}_up"]), dim=1)
        print(f"{tag} alternate_corr fp16: EPE mean {float(e.mean()):.2e} max {float(e.max()):.2e}")
        assert float(e.mean()) <= 2e-3 and float(e.max()) <= 2e-2


def test_raft_alternate_corr_matches_reference_flow_at_1080p(golden):
    """configs[4] end to end at its own resolution: RAFT(alternate_corr=True) on the on-the-fly fp16 corr kernels,
    one 1080x1920 pair ('sintel' padding to 1088x1920, 135 x 240 queries), 12 iterations, against the reference's
    flows for the same pair (tests/golden/raft_e2e_hd.npz: its dense fp32 CPU path -- the reference's alternate corr
    needs a CUDA extension). SURVEY §8(c) fp16 bar: mean EPE <= 2e-3 px, max <= 2e-2 px, on the 1/8-res flow and on
    the full-res flow at stride 8."""
    g = golden("raft_e2e_hd")
    b, h, w, iters, s, seed = (int(v) for v in g["hd1_cfg"])
    img0, img1 = synthetic.synthetic_pair(b, h, w, seed=seed)
    padder = InputPadder(img0.shape, mode=str(g["hd1_mode"]))
    model = RAFT(alternate_corr=True).eval()
    model.load_state_dict(synthetic.synthetic_state_dict(model.state_dict()))
    model = model.to(DEV)
    with torch.inference_mode():
        low, up = model(*(x.to(DEV) for x in padder.pad(img0, img1)), iters=iters, test_mode=True)
    up = padder.unpad(up)[..., ::s, ::s].cpu()
    el = torch.norm(low.float().cpu() - torch.from_numpy(g["hd1_low"]), dim=1)
    eu = torch.norm(up - torch.from_numpy(g["hd1_up"]), dim=1)
    print(f"1080p alternate_corr fp16: EPE low mean {float(el.mean()):.2e} max {float(el.max()):.2e}, "
          f"up mean {float(eu.mean()):.2e} max {float(eu.max()):.2e}")
    assert float(el.mean()) <= 2e-3 and float(el.max()) <= 2e-2
    assert float(eu.mean()) <= 2e-3 and float(eu.max()) <= 2e-2
