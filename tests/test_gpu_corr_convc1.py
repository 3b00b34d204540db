"""The correlation lookup fused into convc1 (csrc/corr_convc1.hip, oflow_corr_lookup_convc1_s32).

Reference: the unfused path's operands -- the NHWC lookup rows (oflow_corr_lookup_tiled_nhwc_f32, itself pinned to the
reference's lookup by tests/test_gpu_parity.py; the fused kernel computes its taps with the same bilinear4 arithmetic)
split into the fp16 hi + lo pair the kernel multiplies -- through a float64 1x1 convolution + ReLU (update.py:120). The
tolerance is test_gpu_conv_s32.py's: |d| <= 2e-6 * sum|x||w| + 1e-6 plus the S32 output's 2^-22 relative rounding.
Also: the fused RAFT forward against the unfused one (NHWC rows -> conv_s32) and against the reference's golden flows.
"""
import math

import pytest
import torch

from optical_flow import _native as N
from model import RAFT, InputPadder, synthetic
from model.utils import coords_grid

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    assert torch.cuda.is_available(), "GPU tests need a ROCm GPU"
    N.load()


def _case(b, h, w, levels, radius, sigma, seed, special=False):
    f1, f2 = synthetic.synthetic_fmaps(b, 256, h, w, stream=seed)
    f1, f2 = f1.to(DEV), f2.to(DEV)
    pyr = N.corr_pyramid_tiled(f1, f2, levels)
    coords = coords_grid(b, h, w) + torch.from_numpy(synthetic.hash_normal(seed + 11, (b, 2, h, w), sigma))
    if special:  # non-finite / huge coordinates (all-zero windows) and exact integer centres
        coords[0, 0, 0, :3] = torch.tensor([float("nan"), float("inf"), 1e9])
        coords[0, :, 1, :5] = torch.round(coords[0, :, 1, :5])
    coords = coords.to(DEV).contiguous()
    g = torch.Generator().manual_seed(seed)
    kk = (2 * radius + 1) ** 2
    conv = torch.nn.Conv2d(levels * kk, 256, 1)
    with torch.no_grad():
        conv.weight.copy_(torch.randn(conv.weight.shape, generator=g) / math.sqrt(levels * kk) * 4.0)
        conv.bias.copy_(torch.randn(256, generator=g) * 0.1)
    return pyr, coords, conv.to(DEV)


def _reference(pyr, coords, conv, radius):
    b, _, h, w = coords.shape
    kk = (2 * radius + 1) ** 2
    rows = torch.empty((b * h * w, len(pyr.levels) * kk), device=DEV)
    N.corr_lookup_tiled_nhwc(pyr, coords, radius, rows)
    hi = rows.half()
    lo = (rows - hi.float()).half()
    x = hi.double() + lo.double()  # the operand the kernel multiplies
    wt = conv.weight.detach().double().view(256, -1)
    y = x @ wt.t() + conv.bias.detach().double()
    bound = x.abs() @ wt.abs().t()
    return torch.relu(y), bound, rows


CASES = [
    # b, h, w, levels, radius, sigma, special
    (2, 55, 128, 4, 4, 3.0, False),  # Sintel 1/8 grid, RAFT's configuration
    (1, 19, 45, 4, 4, 20.0, True),   # ragged query count (855), far-out windows, NaN / inf / huge coords
    (2, 20, 37, 3, 4, 0.0, False),   # integer-free zero-flow centres, 3 levels
    (1, 47, 96, 4, 3, 6.0, False),   # radius 3 (RAFT-small's window), 2 k32 groups per level
    (3, 16, 16, 2, 4, 1.5, False),
]


@pytest.mark.parametrize("b,h,w,levels,radius,sigma,special", CASES)
def test_corr_lookup_convc1_matches_fp64(b, h, w, levels, radius, sigma, special):
    pyr, coords, conv = _case(b, h, w, levels, radius, sigma, seed=b * 100 + h + levels, special=special)
    cw = N.convc1_level_weights(conv, levels, radius)
    out = N.s32_empty(b, h, w, 8, DEV, zero=True)
    N.corr_lookup_convc1(pyr, coords, radius, cw, N.S32Slice(out))
    torch.cuda.synchronize()
    ref, bound, _ = _reference(pyr, coords, conv, radius)
    got = N.s32_to_f32(out, 256).permute(0, 2, 3, 1).reshape(b * h * w, 256).double()
    tol = 2e-6 * bound + 1e-6 + 2.0 ** -22 * ref.abs()
    err = (got - ref).abs()
    assert bool((err <= tol).all()), f"max err {float(err.max()):.3e}, worst ratio {float((err / tol).max()):.2f}"


def test_corr_lookup_convc1_equals_unfused_conv():
    """Fused kernel vs the unfused pair it replaces (NHWC lookup rows -> oflow_conv_s32 OFLOW_IN_F32 -> ReLU): the same
    split operands, summed in another k order (level-padded groups), so equal to fp32 accumulation noise."""
    b, h, w = 2, 55, 128
    pyr, coords, conv = _case(b, h, w, 4, 4, 4.0, seed=5)
    out = N.s32_empty(b, h, w, 8, DEV, zero=True)
    N.corr_lookup_convc1(pyr, coords, 4, N.convc1_level_weights(conv, 4, 4), N.S32Slice(out))
    rows = torch.empty((b * h * w, 324), device=DEV)
    N.corr_lookup_tiled_nhwc(pyr, coords, 4, rows)
    ref = N.s32_empty(b, h, w, 8, DEV, zero=True)
    N.conv_s32(N.F32In(rows, b, h, w), N.ConvWeights(conv.weight, conv.bias, 256), 128, "relu", y0=N.S32Slice(ref))
    torch.cuda.synchronize()
    a, r = N.s32_to_f32(out, 256), N.s32_to_f32(ref, 256)
    assert float((a - r).abs().max()) <= 2e-5 * float(r.abs().max())


def test_corr_lookup_convc1_argument_errors():
    pyr, coords, conv = _case(1, 16, 16, 4, 4, 1.0, seed=3)
    out = N.s32_empty(1, 16, 16, 8, DEV)
    with pytest.raises(RuntimeError):  # weights of another radius
        N.corr_lookup_convc1(pyr, coords, 4, N.convc1_level_weights(torch.nn.Conv2d(4 * 49, 256, 1).to(DEV), 4, 3), N.S32Slice(out))
    with pytest.raises(RuntimeError):  # coords of another batch
        N.corr_lookup_convc1(pyr, coords.repeat(2, 1, 1, 1), 4, N.convc1_level_weights(conv, 4, 4), N.S32Slice(out))


def _raft(fusion: bool):
    model = RAFT().eval()
    model.load_state_dict(synthetic.synthetic_state_dict(model.state_dict()))
    model = model.to(DEV)
    model.lookup_fusion = fusion
    return model


@pytest.mark.parametrize("pairs", [1, 3])
def test_raft_fused_lookup_equals_unfused(pairs):
    img0, img1 = synthetic.synthetic_pair(pairs, 128, 256, seed=4)
    img0, img1 = img0.to(DEV), img1.to(DEV)
    with torch.inference_mode():
        lo_f, up_f = _raft(True)(img0, img1, iters=12, test_mode=True)
        lo_u, up_u = _raft(False)(img0, img1, iters=12, test_mode=True)
    epe = torch.norm(up_f - up_u, dim=1)
    assert float(epe.mean()) <= 1e-5 and float(epe.max()) <= 2e-4, (float(epe.mean()), float(epe.max()))


@pytest.mark.parametrize("fusion", [True, False])
def test_raft_lookup_paths_golden_kitti(golden, fusion):
    """The reference's own KITTI flows (2 pairs: the pair-lane path) with the lookup fused into convc1 and unfused:
    SURVEY §8(c)'s fp32 bar (tests/test_gpu_raft.py runs every golden case with the default, fused)."""
    g = golden("raft_e2e")
    b, h, w, iters, s, seed = (int(v) for v in g["kitti_cfg"])
    img0, img1 = synthetic.synthetic_pair(b, h, w, seed=seed)
    padder = InputPadder(img0.shape, mode=str(g["kitti_mode"]))
    p0, p1 = (x.to(DEV) for x in padder.pad(img0, img1))
    with torch.inference_mode():
        low, up = _raft(fusion)(p0, p1, iters=iters, test_mode=True)
    up = padder.unpad(up)[..., ::s, ::s].cpu()
    epe = torch.norm(up - torch.from_numpy(g["kitti_up"]), dim=1)
    assert float(epe.mean()) <= 1e-4 and float(epe.max()) <= 1e-3, (float(epe.mean()), float(epe.max()))


def test_raft_fused_lanes_deterministic_on_dirty_memory():
    """Every buffer the fused pair-lane forward reads is written first: with the caching allocator's free blocks
    filled with NaN beforehand, three forwards (KITTI grid, 2 pairs = 2 lanes) give finite, identical flows."""
    img0, img1 = synthetic.synthetic_pair(2, 376, 1248, seed=2)
    img0, img1 = img0.to(DEV), img1.to(DEV)
    model = _raft(True)
    outs = []
    for _ in range(3):
        junk = torch.full((512, 1024, 1024), float("nan"), device=DEV)  # 2 GiB of NaN back into the pool
        del junk
        with torch.inference_mode():
            outs.append(model(img0, img1, iters=6, test_mode=True)[1])
        torch.cuda.synchronize()
    for o in outs:
        assert bool(torch.isfinite(o).all())
        assert torch.equal(o, outs[0])


def test_raft_fnet_streams_bit_identical():
    """fnet's two images on two streams (RAFT.fnet_streams) = one 2B batch, bit for bit (instance norm is per image)."""
    img0, img1 = synthetic.synthetic_pair(3, 128, 256, seed=8)
    img0, img1 = img0.to(DEV), img1.to(DEV)
    model = _raft(True)
    outs = []
    for fs in (True, False):
        model.fnet_streams = fs
        with torch.inference_mode():
            outs.append(model(img0, img1, iters=6, test_mode=True)[1])
    assert torch.equal(outs[0], outs[1])
