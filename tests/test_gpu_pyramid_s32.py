"""Split-fp16 correlation pyramid (oflow_corr_pyramid_tiled_s32: the RAFT forward's pyramid from S32 features).

References: the float64 restatement of corr.py:38-54, 79-87 on (a) the ORIGINAL fp32 features -- SURVEY §8(c)'s pyramid
bar, |d| <= 1e-4 + 1e-5 |ref| -- and (b) the S32 operands the kernel sees (hi + lo): there the only errors are the
dropped lo*lo term and fp32 accumulation, bounded by 2^-18 * sum|a||b| / sqrt(C) + 1e-7 per element (fp32 accumulation over C terms). Level l + 1 must
equal ATen's avg_pool2d of level l bit for bit (pooling is the fp32 kernel's epilogue code), and RAFT with the split
pyramid must stay on the reference's flows (tests/test_gpu_raft.py runs the goldens with it; here: vs the fp32 pyramid).
"""
import pytest
import torch
import torch.nn.functional as F

from optical_flow import _native as N
from model import RAFT, synthetic

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    assert torch.cuda.is_available(), "GPU tests need a ROCm GPU"
    N.load()


def _levels64(f1, f2, L):
    b, c, h, w = f1.shape
    corr = torch.einsum("bci,bcj->bij", f1.reshape(b, c, -1).double(), f2.reshape(b, c, -1).double()) / c ** 0.5
    lv = [corr.reshape(b * h * w, 1, h, w)]
    for _ in range(L - 1):
        lv.append(F.avg_pool2d(lv[-1], 2, stride=2))
    return lv


SHAPES = [(2, 256, 55, 128, 4), (1, 256, 47, 156, 4), (3, 64, 16, 20, 3), (1, 128, 13, 45, 2), (2, 256, 9, 33, 1)]


@pytest.mark.parametrize("b,c,h,w,L", SHAPES)
def test_pyramid_s32_matches_fp64(b, c, h, w, L):
    f1, f2 = synthetic.synthetic_fmaps(b, c, h, w, stream=h + w)
    s1, s2 = N.s32_from_f32(f1.to(DEV)), N.s32_from_f32(f2.to(DEV))
    pyr = N.corr_pyramid_tiled_s32(s1, s2, L)
    got = [pyr.untile(l).cpu().double() for l in range(L)]
    ref = _levels64(f1, f2, L)  # the original fp32 features
    r1 = N.s32_to_f32(s1, c).cpu()
    r2 = N.s32_to_f32(s2, c).cpu()
    refs = _levels64(r1, r2, L)  # the split operands
    bound = _levels64(r1.abs(), r2.abs(), L)
    for l in range(L):
        err = (got[l] - ref[l]).abs()
        assert bool((err <= 1e-4 + 1e-5 * ref[l].abs()).all()), f"level {l}: max err {float(err.max()):.3e}"
        err_s = (got[l] - refs[l]).abs()
        assert bool((err_s <= 2.0 ** -18 * bound[l] + 1e-7).all()), f"level {l} vs split operands: {float(err_s.max()):.3e}"
    for l in range(1, L):  # pooling: ATen's avg_pool2d of the level above, bit for bit
        assert torch.equal(got[l].float(), F.avg_pool2d(got[l - 1].float(), 2, stride=2))


def test_pyramid_s32_rejects_bad_input():
    f = N.s32_empty(1, 8, 8, 2, DEV)
    with pytest.raises(RuntimeError):
        N.corr_pyramid_tiled_s32(f, N.s32_empty(1, 8, 9, 2, DEV), 2)
    with pytest.raises(RuntimeError):
        N.corr_pyramid_tiled_s32(f.float(), f.float(), 2)


def test_raft_split_corr_equals_fp32_corr():
    img0, img1 = synthetic.synthetic_pair(2, 256, 384, seed=6)
    img0, img1 = img0.to(DEV), img1.to(DEV)
    model = RAFT().eval()
    model.load_state_dict(synthetic.synthetic_state_dict(model.state_dict()))
    model = model.to(DEV)
    outs = []
    for split in (True, False):
        model.split_corr = split
        with torch.inference_mode():
            outs.append(model(img0, img1, iters=12, test_mode=True)[1])
    epe = torch.norm(outs[0] - outs[1], dim=1)
    assert float(epe.mean()) <= 1e-5 and float(epe.max()) <= 2e-4, (float(epe.mean()), float(epe.max()))
