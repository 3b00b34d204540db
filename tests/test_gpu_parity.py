"""Parity of the gfx950 HIP path (through the C ABI of liboflow_hip.so) against the oracle and the goldens the
reference produced. Tolerances: corr pyramid fp32 |d| <= 1e-4 + 1e-5|ref|; lookup |d| <= 1e-4;
warp / grid_sample: bit-exact (every mode and padding: the kernel evaluates ATen's CPU arithmetic, fused
multiply-adds included -- tools/exp/gridsample_emul.py pins that model against torch);
end-to-end mean EPE <= 1e-4 px... see the individual tests.
"""
import math

import numpy as np
import pytest
import torch
import torch.nn.functional as F

import optical_flow
from model import CorrBlock, bilinear_sampler, synthetic
from model.utils import coords_grid
from optical_flow import _native
from oracle import corr as ocorr
from oracle import operator as oop

pytestmark = pytest.mark.gpu
# the warp / grid_sample goldens and the live oracle run ATen's AVX512 CPU kernels; another host vector ISA may
# contract differently, so a live comparison on such a host allows ulp-level noise (1e-5 of the value range)
_EXACT_CPU = torch.backends.cpu.get_cpu_capability() == "AVX512"


def _warp_close(got, ref, what):
    err = (got - ref).abs().max().item() if got.numel() else 0.0
    if _EXACT_CPU:
        assert err == 0.0, (what, err)
    else:
        assert err <= 1e-5 * max(1.0, ref.abs().max().item()), (what, err)
DEV = torch.device("cuda", 0)


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    assert torch.cuda.is_available(), "GPU tests need a ROCm GPU"
    _native.load()


def _assert_pyr(got, ref, what):
    ref = np.asarray(ref)
    got = got.detach().cpu().numpy()
    assert got.shape == ref.shape, (what, got.shape, ref.shape)
    err = np.abs(got - ref)
    tol = 1e-4 + 1e-5 * np.abs(ref)
    assert np.all(err <= tol), f"{what}: max err {err.max()} (worst excess {(err - tol).max()})"


# ----------------------------------------------------------------------------------------------------------
# correlation pyramid
# ----------------------------------------------------------------------------------------------------------
@pytest.mark.parametrize("tag", ["a", "b"])
def test_pyramid_matches_reference_goldens(golden, tag):
    g = golden("corr_small")
    b, c, h, w = (int(v) for v in g[f"{tag}_shape"])
    f1, f2 = synthetic.synthetic_fmaps(b, c, h, w, stream=int(g[f"{tag}_stream"]))
    cb = CorrBlock(f1.to(DEV), f2.to(DEV), num_levels=4, radius=4)
    for lvl in range(4):
        _assert_pyr(cb.corr_pyramid[lvl], g[f"{tag}_pyr{lvl}"], f"{tag} level {lvl}")


@pytest.mark.parametrize(
    "shape,levels",
    [
        ((1, 256, 23, 37), 4),  # W % 4 != 0: scalar staging path, ragged tiles
        ((2, 64, 16, 20), 4),  # C = 64
        ((1, 100, 17, 19), 3),  # sqrt(C) = 10, not a power of two: true division
        ((1, 256, 33, 70), 6),  # levels >= 4 through the stand-alone pooling kernel
        ((3, 256, 9, 12), 1),
        ((1, 7, 31, 64), 2),  # C not a multiple of the 16-channel stage
    ],
)
def test_pyramid_matches_oracle_shapes(shape, levels):
    b, c, h, w = shape
    f1, f2 = synthetic.synthetic_fmaps(b, c, h, w, stream=31 + c)
    ref = ocorr.corr_pyramid(f1, f2, levels)
    got = _native.corr_pyramid(f1.to(DEV), f2.to(DEV), levels)
    for lvl in range(levels):
        _assert_pyr(got[lvl], ref[lvl].numpy(), f"{shape} level {lvl}")


def test_corr_staticmethod_and_views():
    f1, f2 = synthetic.synthetic_fmaps(2, 256, 16, 24, stream=3)
    vol = CorrBlock.corr(f1.to(DEV), f2.to(DEV))
    assert vol.shape == (2, 16, 24, 1, 16, 24)
    _assert_pyr(vol, ocorr.corr_volume(f1, f2).numpy(), "corr volume")


def test_pyramid_exact_properties():
    """Bit-exact, size-independent properties at a Sintel-size shape (55 x 128, batch 2):
    symmetry corr(f1,f2)[i,j] == corr(f2,f1)[j,i] (same k-ordered fp32 fma chain), linearity under a power of
    two, and every pooled level == avg_pool2d(level above) computed by ATen on the GPU."""
    f1, f2 = synthetic.synthetic_fmaps(2, 256, 55, 128, stream=41)
    f1, f2 = f1.to(DEV), f2.to(DEV)
    p = _native.corr_pyramid(f1, f2, 4)
    pt = _native.corr_pyramid(f2, f1, 1)[0]
    n = 55 * 128
    a = p[0].view(2, n, n)
    assert torch.equal(a, pt.view(2, n, n).transpose(1, 2))
    p2 = _native.corr_pyramid(2 * f1, f2, 1)[0]
    assert torch.equal(p2, 2 * p[0])
    for lvl in range(1, 4):
        assert torch.equal(p[lvl], F.avg_pool2d(p[lvl - 1], 2, stride=2)), lvl


# ----------------------------------------------------------------------------------------------------------
# lookup
# ----------------------------------------------------------------------------------------------------------
def test_lookup_matches_reference_goldens(golden):
    g = golden("corr_small")
    for tag in ("a", "b"):
        pyr = [torch.from_numpy(g[f"{tag}_pyr{lvl}"]).to(DEV) for lvl in range(4)]
        for k in [k for k in g if k.startswith(f"{tag}_coords_") and k != "a_coords_r2"]:
            out = _native.corr_lookup(pyr, torch.from_numpy(g[k]).to(DEV), 4).cpu().numpy()
            ref = g[k.replace("coords", "lookup")]
            err = np.abs(out - ref).max()
            assert err <= 1e-4, (k, err)
    pyr3 = [torch.from_numpy(g[f"a_pyr{lvl}"]).to(DEV) for lvl in range(3)]
    out = _native.corr_lookup(pyr3, torch.from_numpy(g["a_coords_r2"]).to(DEV), 2).cpu().numpy()
    assert np.abs(out - g["a_lookup_r2_l3"]).max() <= 1e-4


@pytest.mark.parametrize("radius", [0, 1, 3, 4, 7])
@pytest.mark.parametrize("sigma", [0.0, 2.5, 30.0])
def test_lookup_matches_oracle(radius, sigma):
    b, h, w = 2, 19, 26
    f1, f2 = synthetic.synthetic_fmaps(b, 64, h, w, stream=5)
    pyr = ocorr.corr_pyramid(f1, f2, 4)
    coords = ocorr.coords_grid(b, h, w) + torch.from_numpy(synthetic.hash_normal(70 + radius, (b, 2, h, w), sigma))
    ref = ocorr.corr_lookup(pyr, coords, radius)
    got = _native.corr_lookup([p.to(DEV) for p in pyr], coords.to(DEV), radius)
    assert got.shape == ref.shape
    assert (got.cpu() - ref).abs().max().item() <= 1e-4


def test_lookup_window_channel_order_q1():
    vol = torch.zeros(1, 1, 16, 16)
    vol[0, 0, 8 + 3, 8 + 1] = 1.0
    out = _native.corr_lookup([vol.to(DEV)], torch.tensor([8.0, 8.0]).view(1, 2, 1, 1).to(DEV), 4)
    assert int(out.view(-1).argmax()) == 5 * 9 + 7 and float(out.sum()) == 1.0


def test_lookup_integer_coords_are_exact_gathers():
    """wx = wy = 0 -> every output is exactly one pyramid value (or 0 outside)."""
    f1, f2 = synthetic.synthetic_fmaps(1, 32, 16, 16, stream=9)
    pyr = [p.to(DEV) for p in ocorr.corr_pyramid(f1, f2, 2)]
    coords = ocorr.coords_grid(1, 16, 16).to(DEV)
    out = _native.corr_lookup(pyr, coords, 2).cpu()
    p0 = pyr[0].cpu().view(16, 16, 16, 16)
    for q, (y, x) in enumerate([(0, 0), (7, 9), (15, 15)]):
        for i in range(5):
            for j in range(5):
                yy, xx = y + j - 2, x + i - 2
                exp = p0[y, x, yy, xx] if (0 <= yy < 16 and 0 <= xx < 16) else 0.0
                assert out[0, i * 5 + j, y, x] == exp


def test_lookup_non_finite_and_huge_coords_give_zero():
    f1, f2 = synthetic.synthetic_fmaps(1, 16, 16, 16, stream=2)
    pyr = [p.to(DEV) for p in ocorr.corr_pyramid(f1, f2, 4)]
    coords = ocorr.coords_grid(1, 16, 16)
    coords[0, 0, 0, 0] = float("nan")
    coords[0, 1, 0, 1] = float("inf")
    coords[0, 0, 0, 2] = 1e9
    coords[0, 0, 0, 3] = -5e6
    out = _native.corr_lookup(pyr, coords.to(DEV), 4).cpu()
    assert torch.all(out[0, :, 0, :4] == 0)
    assert torch.isfinite(out).all()


def test_lookup_rejects_tiny_levels_q3():
    f1, f2 = synthetic.synthetic_fmaps(1, 16, 8, 12, stream=2)
    cb = CorrBlock(f1.to(DEV), f2.to(DEV))  # levels 8x12 .. 1x1
    with pytest.raises(ValueError, match="2 pixels"):
        cb(coords_grid(1, 8, 12, device=DEV))


def test_pyramid_full_size_fp64_spot_check():
    """configs[1] shape (B=4, C=256, 128 x 128): levels 0-3 of the HIP pyramid (the tiled layout CorrBlock uses,
    untiled) at 320 random queries against a float64 restatement of corr.py:38-54 (dot products / sqrt(C), floor 2x2
    average pools), within SURVEY §8(c)'s fp32 tolerance |d| <= 1e-4 + 1e-5 |ref|."""
    b, c, h, w = 4, 256, 128, 128
    f1, f2 = synthetic.synthetic_fmaps(b, c, h, w, stream=17)
    cb = CorrBlock(f1.to(DEV), f2.to(DEV))
    got = [t.cpu().numpy() for t in cb.corr_pyramid]
    a = f1.double().numpy().reshape(b, c, h * w)
    m = f2.double().numpy().reshape(b, c, h * w)
    qs = np.random.default_rng(1).integers(0, b * h * w, 320)
    worst = 0.0
    for q in qs:
        bi, i = divmod(int(q), h * w)
        lvl = (a[bi, :, i] @ m[bi] / math.sqrt(c)).reshape(h, w)
        for l in range(4):
            if l:
                hh, ww = lvl.shape[0] // 2, lvl.shape[1] // 2
                lvl = lvl[: 2 * hh, : 2 * ww].reshape(hh, 2, ww, 2).mean(axis=(1, 3))
            d = np.abs(got[l][q, 0] - lvl)
            assert (d <= 1e-4 + 1e-5 * np.abs(lvl)).all(), (q, l, float(d.max()))
            worst = max(worst, float(d.max()))
    print(f"configs[1] pyramid vs fp64: max |d| {worst:.2e} over 320 queries x 4 levels")


def test_lookup_full_size_spot_check():
    """Config #2 shape (B=4, 128 x 128, C=256): spot-check 256 queries against the float64 oracle."""
    b, h, w = 4, 128, 128
    f1, f2 = synthetic.synthetic_fmaps(b, 256, h, w, stream=13)
    cb = CorrBlock(f1.to(DEV), f2.to(DEV))
    coords = coords_grid(b, h, w) + torch.from_numpy(synthetic.hash_normal(14, (b, 2, h, w), 4.0))
    out = cb(coords.to(DEV)).cpu()
    rng = np.random.default_rng(0)
    qs = rng.integers(0, b * h * w, 256)
    n = h * w
    for q in qs:
        bi, pix = divmod(int(q), n)
        pyr = [cb.corr_pyramid[l][q : q + 1].cpu().numpy() for l in range(4)]
        c = coords[bi : bi + 1, :, pix // w : pix // w + 1, pix % w : pix % w + 1].numpy()
        ref = ocorr.corr_lookup_f64(pyr, c, 4)[0, :, 0, 0]
        assert np.abs(out[bi, :, pix // w, pix % w].numpy() - ref).max() <= 1e-4


# ----------------------------------------------------------------------------------------------------------
# warp / grid_sample
# ----------------------------------------------------------------------------------------------------------
def test_warp_reference_unit_tests_exact():
    """tests/operator/test_operator.py:6-38 of the reference, bit-exact."""
    img = torch.tensor([[[1.0, 2.0]]]).unsqueeze(0).to(DEV)
    flow = torch.tensor([[[1.0, 0.0]], [[0.0, 0.0]]]).unsqueeze(0).to(DEV)
    assert torch.equal(optical_flow.warp(img, optical_flow.normalize(flow)).cpu(), torch.tensor([[[[2.0, 2.0]]]]))
    img = torch.tensor([[[1.0], [2.0]]]).unsqueeze(0).to(DEV)
    flow = torch.tensor([[[0.0], [0.0]], [[1.0], [0.0]]]).unsqueeze(0).to(DEV)
    assert torch.equal(optical_flow.warp(img, optical_flow.normalize(flow)).cpu(), torch.tensor([[[[2.0], [2.0]]]]))


def test_warp_matches_reference_goldens(golden):
    g = golden("warp_small")
    frame, flow = torch.from_numpy(g["frame"]).to(DEV), torch.from_numpy(g["flow"]).to(DEV)
    for key in g:
        if key.startswith("warp_") and key != "warp_default":
            _, mode, pad, ac = key.split("_")
            out = optical_flow.warp(frame, flow, mode, pad, bool(int(ac))).cpu().numpy()
            np.testing.assert_array_equal(out, g[key], err_msg=key)  # the reference's own outputs, bit for bit
    np.testing.assert_array_equal(optical_flow.warp(frame, flow).cpu().numpy(), g["warp_default"])
    fp = torch.from_numpy(g["flow_px"]).to(DEV)
    out = optical_flow.integrate(fp, 0.5 * fp, -0.25 * fp).cpu().numpy()
    np.testing.assert_array_equal(out, g["integrate_3"])


@pytest.mark.parametrize("mode", ["bilinear", "nearest", "bicubic"])
@pytest.mark.parametrize("pad", ["zeros", "border", "reflection"])
@pytest.mark.parametrize("ac", [False, True])
def test_warp_matches_oracle_sintel_frame(mode, pad, ac):
    img0, _ = synthetic.synthetic_pair(2, 109, 256, seed=4)
    flow = oop.normalize(torch.from_numpy(synthetic.hash_normal(6, (2, 2, 109, 256), 8.0)))
    ref = oop.warp(img0, flow, mode, pad, ac)
    got = optical_flow.warp(img0.to(DEV), flow.to(DEV), mode, pad, ac).cpu()
    _warp_close(got, ref, (mode, pad, ac))


@pytest.mark.parametrize("width", [331, 332])
@pytest.mark.parametrize("sigma", [0.0, 2.0, 40.0, 300.0])
@pytest.mark.parametrize("pad", ["zeros", "border", "reflection"])
def test_warp_bilinear_staged_and_direct_tiles(sigma, pad, width):
    """The bilinear warp stages a tile's source box in LDS when its taps fit (small sigma) and gathers directly
    otherwise (sigma 300 px; single far-out pixels inside otherwise staged tiles; rows that are not 16-B multiples,
    width 331): both against the oracle."""
    img0, _ = synthetic.synthetic_pair(2, 150, width, seed=5)
    px = torch.from_numpy(synthetic.hash_normal(12, (2, 2, 150, width), sigma))
    px[0, :, 7, 5] = torch.tensor([5000.0, -3000.0])  # one pixel far outside the frame
    for ac in (False, True):
        flow = oop.normalize(px)
        ref = oop.warp(img0, flow, "bilinear", pad, ac)
        got = optical_flow.warp(img0.to(DEV), flow.to(DEV), "bilinear", pad, ac).cpu()
        _warp_close(got, ref, (sigma, pad, ac))


@pytest.mark.parametrize("c,h,w,sigma", [(1, 77, 132, 8.0), (3, 436, 1024, 8.0), (4, 50, 64, 20.0), (3, 70, 64, 20.0), (2, 33, 200, 0.0),
                                           (3, 130, 96, 60.0)])
@pytest.mark.parametrize("pad", ["zeros", "border", "reflection"])
def test_warp_strip_kernel_equals_tile_kernel(c, h, w, sigma, pad):
    """The strip-walking warp (64-column strips, 16-row steps, an LDS ring of +-28 px; taps outside it gathered from
    global memory: sigma 20 / 60) = the per-tile staged kernel (oflow_exp_set_warp_strip(0)), bit for bit; ragged
    heights (segments ending mid-step), C = 1..4, the SURVEY warp workload's frame size; and = the oracle."""
    import ctypes
    g = torch.Generator().manual_seed(c * 1000 + h)
    img = (torch.rand(2, c, h, w, generator=g) * 255).floor()
    px = torch.from_numpy(synthetic.hash_normal(13 + c, (2, 2, h, w), sigma)) if sigma > 0 else torch.zeros(2, 2, h, w)
    flow = oop.normalize(px)
    lib = _native.load()
    lib.oflow_exp_set_warp_strip.argtypes = [ctypes.c_int]
    outs = []
    for on in (1, 0):
        lib.oflow_exp_set_warp_strip(on)
        try:
            outs.append(optical_flow.warp(img.to(DEV), flow.to(DEV), "bilinear", pad, False).cpu())
        finally:
            lib.oflow_exp_set_warp_strip(1)
    assert torch.equal(outs[0], outs[1])
    _warp_close(outs[0], oop.warp(img, flow, "bilinear", pad, False), (c, h, w, sigma, pad))


def test_grid_sample_and_bilinear_sampler_match_oracle():
    img = torch.from_numpy(synthetic.hash_normal(8, (6, 3, 20, 30), 1.0))
    coords = torch.from_numpy(synthetic.hash_normal(9, (6, 7, 5, 2), 12.0)) + 12.0
    ref = ocorr.bilinear_sampler(img, coords)
    got = bilinear_sampler(img.to(DEV), coords.to(DEV)).cpu()
    assert (got - ref).abs().max().item() <= 1e-5
    out, mask = bilinear_sampler(img.to(DEV), coords.to(DEV), mask=True)
    assert mask.shape == (6, 7, 5, 1)
    grid = torch.from_numpy(synthetic.hash_normal(10, (2, 9, 11, 2), 0.8))
    x = torch.from_numpy(synthetic.hash_normal(11, (2, 4, 13, 17), 1.0))
    for mode in ("bilinear", "nearest", "bicubic"):
        for pad in ("zeros", "border", "reflection"):
            for ac in (False, True):
                r = F.grid_sample(x, grid, mode=mode, padding_mode=pad, align_corners=ac)
                gg = _native.grid_sample(x.to(DEV), grid.to(DEV), mode, pad, ac).cpu()
                _warp_close(gg, r, (mode, pad, ac))


def test_ops_follow_the_current_stream():
    f1, f2 = synthetic.synthetic_fmaps(1, 256, 24, 32, stream=1)
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        cb = CorrBlock(f1.to(DEV), f2.to(DEV))
        out = cb(coords_grid(1, 24, 32, device=DEV))
    s.synchronize()
    ref = ocorr.corr_lookup(ocorr.corr_pyramid(f1, f2, 4), ocorr.coords_grid(1, 24, 32), 4)
    assert (out.cpu() - ref).abs().max().item() <= 1e-4


# ----------------------------------------------------------------------------------------------------------
# tiled layout (what CorrBlock uses): must be a pure re-addressing of the canonical kernels' results
# ----------------------------------------------------------------------------------------------------------
@pytest.mark.parametrize("shape,levels", [((1, 256, 23, 37), 4), ((2, 64, 16, 20), 4), ((1, 256, 33, 70), 6), ((2, 256, 55, 128), 4)])
def test_tiled_pyramid_untiles_to_canonical_bit_exact(shape, levels):
    b, c, h, w = shape
    f1, f2 = synthetic.synthetic_fmaps(b, c, h, w, stream=61 + c)
    f1, f2 = f1.to(DEV), f2.to(DEV)
    tp = _native.corr_pyramid_tiled(f1, f2, levels)
    cp = _native.corr_pyramid(f1, f2, levels)
    for lvl in range(levels):
        assert torch.equal(tp.untile(lvl), cp[lvl]), lvl


@pytest.mark.parametrize("radius", [0, 2, 4, 7])
@pytest.mark.parametrize("sigma", [0.0, 4.0, 40.0])
def test_tiled_lookup_equals_canonical_lookup(radius, sigma):
    b, h, w = 2, 47, 156  # KITTI 1/8 grid: W_l not multiples of 8 at any level
    f1, f2 = synthetic.synthetic_fmaps(b, 256, h, w, stream=63)
    f1, f2 = f1.to(DEV), f2.to(DEV)
    coords = (coords_grid(b, h, w) + torch.from_numpy(synthetic.hash_normal(64, (b, 2, h, w), sigma))).to(DEV)
    tp = _native.corr_pyramid_tiled(f1, f2, 4)
    cp = _native.corr_pyramid(f1, f2, 4)
    assert torch.equal(_native.corr_lookup_tiled(tp, coords, radius), _native.corr_lookup(cp, coords, radius))


def test_corrblock_pyramid_attribute_semantics():
    """corr_pyramid reads as the reference's list; after access (or assignment) lookups follow that list."""
    f1, f2 = synthetic.synthetic_fmaps(1, 64, 16, 16, stream=65)
    cb = CorrBlock(f1.to(DEV), f2.to(DEV))
    coords = coords_grid(1, 16, 16, device=DEV) + 0.5
    before = cb(coords)
    pyr = cb.corr_pyramid
    assert [tuple(p.shape) for p in pyr] == [(256, 1, 16, 16), (256, 1, 8, 8), (256, 1, 4, 4), (256, 1, 2, 2)]
    assert torch.equal(cb(coords), before)
    pyr[0].zero_()
    after = cb(coords)
    assert torch.all(after[:, :81] == 0) and torch.equal(after[:, 81:], before[:, 81:])
    cb.corr_pyramid = [p * 2 for p in pyr]
    assert torch.equal(cb(coords)[:, 81:], 2 * before[:, 81:])


def test_inference_layouts_refuse_autograd_inputs():
    """The tiled / fp16 layouts have no autograd formula: an input that requires grad raises instead of silently
    dropping the graph; the canonical ops (corr_pyramid / corr_lookup / grid_warp) differentiate instead."""
    f = torch.randn(1, 8, 16, 16, device=DEV, requires_grad=True)
    with pytest.raises(RuntimeError, match="requires grad"):
        _native.corr_pyramid_tiled(f, f.detach(), 1)
    with pytest.raises(RuntimeError, match="requires grad"):
        _native.otf_prepare(torch.randn(1, 32, 16, 16, device=DEV, requires_grad=True), torch.randn(1, 32, 16, 16, device=DEV), 1)
    levels = _native.corr_pyramid(f, f.detach(), 1)
    assert levels[0].requires_grad
    frame = torch.rand(1, 3, 8, 8, device=DEV, requires_grad=True)
    flow = torch.zeros(1, 2, 8, 8, device=DEV)
    assert _native.grid_warp(frame, flow, "bilinear", "border", False).requires_grad
    with torch.no_grad():
        assert optical_flow.warp(frame, flow).shape == frame.shape


@pytest.mark.parametrize("ac", [False, True])
@pytest.mark.parametrize("mode", ["bilinear", "nearest", "bicubic"])
@pytest.mark.parametrize("pad", ["zeros", "border", "reflection"])
def test_warp_autograd_matches_oracle(pad, mode, ac):
    """optical_flow.warp under autograd: HIP forward, native backward (warp_backward.hip) -- frame and flow gradients
    equal the reference operator's (operator.py:8-56) differentiated on the CPU, every mode / padding / align_corners,
    with flows that push taps past every border."""
    img0, _ = synthetic.synthetic_pair(2, 40, 64, seed=9)
    flow = oop.normalize(torch.from_numpy(synthetic.hash_normal(13, (2, 2, 40, 64), 6.0)))
    r = torch.from_numpy(synthetic.hash_normal(14, (2, 3, 40, 64), 1.0))
    a_f, a_w = img0.clone().requires_grad_(), flow.clone().requires_grad_()
    (oop.warp(a_f, a_w, mode, pad, ac) * r).sum().backward()
    d_f, d_w = img0.to(DEV).requires_grad_(), flow.to(DEV).requires_grad_()
    (optical_flow.warp(d_f, d_w, mode, pad, ac) * r.to(DEV)).sum().backward()
    gf = float(a_f.grad.abs().max())
    assert float((d_f.grad.cpu() - a_f.grad).abs().max()) <= 1e-5 * gf + 1e-4
    gw = float(a_w.grad.abs().max())
    assert float((d_w.grad.cpu() - a_w.grad).abs().max()) <= 1e-3 * gw + 1e-3


@pytest.mark.parametrize("mode", ["bilinear", "nearest", "bicubic"])
@pytest.mark.parametrize("pad", ["zeros", "border", "reflection"])
def test_grid_sample_autograd_matches_oracle(pad, mode):
    """torch.ops.oflow.grid_sample (bilinear_sampler's explicit grid, utils.py:64-80) under autograd with the native
    backward vs F.grid_sample differentiated on the CPU: input and grid gradients, an output size other than the
    input's, grid values past [-1, 1]."""
    g = torch.Generator().manual_seed(3)
    x = torch.randn(2, 5, 17, 23, generator=g)
    grid = torch.rand(2, 11, 13, 2, generator=g) * 2.6 - 1.3
    r = torch.randn(2, 5, 11, 13, generator=g)
    a_x, a_g = x.clone().requires_grad_(), grid.clone().requires_grad_()
    (torch.nn.functional.grid_sample(a_x, a_g, mode=mode, padding_mode=pad, align_corners=True) * r).sum().backward()
    d_x, d_g = x.to(DEV).requires_grad_(), grid.to(DEV).requires_grad_()
    out = torch.ops.oflow.grid_sample(d_x, d_g, _native.INTERP[mode], _native.PADDING[pad], True)
    (out * r.to(DEV)).sum().backward()
    assert float((d_x.grad.cpu() - a_x.grad).abs().max()) <= 1e-5 * float(a_x.grad.abs().max()) + 1e-5
    assert float((d_g.grad.cpu() - a_g.grad).abs().max()) <= 1e-4 * float(a_g.grad.abs().max()) + 1e-4


@pytest.mark.parametrize("b,c,n", [(2, 256, 1000), (1, 32, 792), (3, 70, 130)])
def test_fmap_gradient_gemms_match_fp64(b, c, n):
    """The fmap gradients of the correlation (corr.py:85 transposed) on fp32 MFMA (oflow_corr_fmap_grad_f32 through
    corr_pyramid_backward, one level) vs float64: grad_f1 = f2 . G^T / sqrt(C), grad_f2 = f1 . G / sqrt(C); ragged
    64-tiles in C and N."""
    g = torch.Generator().manual_seed(c + n)
    h, w = 1, n
    f1 = torch.randn(b, c, h, w, generator=g)
    f2 = torch.randn(b, c, h, w, generator=g)
    g0 = torch.randn(b * n, 1, h, w, generator=g)
    g1, g2 = torch.ops.oflow.corr_pyramid_backward([g0.to(DEV)], f1.to(DEV), f2.to(DEV))
    G = g0.double().view(b, n, n)
    s = 1.0 / math.sqrt(c)
    r1 = torch.bmm(f2.double().view(b, c, n), G.transpose(1, 2)) * s
    r2 = torch.bmm(f1.double().view(b, c, n), G) * s
    bound1 = torch.bmm(f2.double().abs().view(b, c, n), G.abs().transpose(1, 2)) * s
    bound2 = torch.bmm(f1.double().abs().view(b, c, n), G.abs()) * s
    assert bool(((g1.cpu().double().view(b, c, n) - r1).abs() <= 2e-5 * bound1 + 1e-6).all())
    assert bool(((g2.cpu().double().view(b, c, n) - r2).abs() <= 2e-5 * bound2 + 1e-6).all())


@pytest.mark.parametrize("ac", [False, True])
@pytest.mark.parametrize("pad", ["border", "reflection", "zeros"])
def test_grid_sample_bicubic_far_out_grid_backward(pad, ac):
    """Bicubic backward with grid values of about +-1e7 (tap coordinates far past 2^20): under border / reflection
    padding every tap is padded from its float coordinate, so the input gradient lands on the border / reflected pixels
    as ATen's grid_sampler_2d_backward puts it (the forward samples those pixels too); zeros padding drops them."""
    g = torch.Generator().manual_seed(17)
    x = torch.randn(1, 3, 9, 12, generator=g)
    grid = torch.rand(1, 6, 7, 2, generator=g) * 2.0 - 1.0
    grid[0, :3, :, 0] = 1e7
    grid[0, 3:, :4, 1] = -1e7
    grid[0, 5, 6] = torch.tensor([-3e7, 2e7])
    r = torch.randn(1, 3, 6, 7, generator=g)
    a_x = x.clone().requires_grad_()
    (torch.nn.functional.grid_sample(a_x, grid, mode="bicubic", padding_mode=pad, align_corners=ac) * r).sum().backward()
    d_x = x.to(DEV).requires_grad_()
    out = torch.ops.oflow.grid_sample(d_x, grid.to(DEV), _native.INTERP["bicubic"], _native.PADDING[pad], ac)
    (out * r.to(DEV)).sum().backward()
    ref = a_x.grad
    assert float(ref.abs().max()) > 0 or pad == "zeros"
    assert float((d_x.grad.cpu() - ref).abs().max()) <= 1e-5 * float(ref.abs().max()) + 1e-5


def test_warp_backward_forms_only_the_wanted_gradient():
    """needs_input_grad reaches the native backward (output_mask): a frame without gradient gets no frame gradient
    (no zero fill, no atomics), and the flow gradient equals the one computed with both outputs."""
    img0, _ = synthetic.synthetic_pair(1, 24, 40, seed=3)
    flow = oop.normalize(torch.from_numpy(synthetic.hash_normal(15, (1, 2, 24, 40), 4.0)))
    r = torch.from_numpy(synthetic.hash_normal(16, (1, 3, 24, 40), 1.0)).to(DEV)
    f = img0.to(DEV)
    w1 = flow.to(DEV).requires_grad_()
    (optical_flow.warp(f, w1) * r).sum().backward()
    f2, w2 = f.clone().requires_grad_(), flow.to(DEV).requires_grad_()
    (optical_flow.warp(f2, w2) * r).sum().backward()
    assert torch.equal(w1.grad, w2.grad)
    go = r.contiguous()
    gf, gw = torch.ops.oflow.grid_warp_backward(go, f, w1.detach(), 0, 1, False, [False, True])
    assert gf.numel() == 0 and torch.equal(gw, w2.grad)
    gf, gw = torch.ops.oflow.grid_warp_backward(go, f, w1.detach(), 0, 1, False, [True, False])
    assert gw.numel() == 0 and torch.allclose(gf, f2.grad, rtol=1e-5, atol=1e-5)  # fp32 atomics: order varies
