"""Split-fp16 ("S32") update-block kernels (csrc/conv_s32.hip, s32_io.hip) through the C ABI, against PyTorch.

Reference for every convolution: ``F.conv2d`` in float64 on the exact operands the kernel sees (input = hi + lo of
the S32 tensor, fp32 weights), plus the plain PyTorch fp32 convolution on the GPU. Tolerance: the kernel's error
comes from representing weights and activations with 22 significant bits and fp32 accumulation; the bound used is
|d| <= 2e-6 * sum|x||w| (the per-output absolute-product sum, computed by a float64 convolution of |x| and |w|)
+ 1e-6, i.e. a few fp32 roundings of the largest partial sums. Integer exactness: with small-integer operands
(exact in fp16) the result must be exact, which pins the MFMA operand/accumulator lane maps (A = I checks with an
asymmetric B, cdna_hip_programming.md §3).
"""
import math

import pytest
import torch
import torch.nn.functional as F

from optical_flow import _native as N
from model.corr import CorrBlock
from model.utils import coords_grid

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    assert torch.cuda.is_available(), "GPU tests need a ROCm GPU"
    N.load()


def _ref(x, w, b, kh, kw):
    pad = (kh // 2, kw // 2)
    y = F.conv2d(x.double(), w.double(), None if b is None else b.double(), padding=pad)
    bound = F.conv2d(x.double().abs(), w.double().abs(), None, padding=pad)
    return y, bound


def _act(y, act):
    return {"none": y, "relu": torch.relu(y), "sigmoid": torch.sigmoid(y), "tanh": torch.tanh(y)}[act]


CASES = [
    # kh, kw, cin, n, block_n, B, H, W
    (1, 1, 352, 256, 128, 2, 13, 45),
    (3, 3, 256, 192, 64, 2, 13, 45),
    (3, 3, 128, 64, 64, 1, 7, 33),
    (3, 3, 256, 126, 128, 2, 9, 40),
    (3, 3, 256, 2, 32, 2, 11, 70),
    (1, 5, 384, 256, 128, 2, 6, 37),
    (5, 1, 384, 128, 128, 2, 10, 31),
    (1, 1, 100, 96, 32, 1, 5, 64),
    (3, 3, 128, 256, 128, 8, 55, 128),
]


@pytest.mark.parametrize("kh,kw,cin,n,bn,b,h,w", CASES)
def test_conv_s32_matches_fp64(kh, kw, cin, n, bn, b, h, w):
    g = torch.Generator().manual_seed(kh * 1000 + cin + n)
    x = (torch.randn(b, cin, h, w, generator=g) * 1.5).to(DEV)
    wt = (torch.randn(n, cin, kh, kw, generator=g) / math.sqrt(cin * kh * kw)).to(DEV)
    bias = torch.randn(n, generator=g).to(DEV)
    xs = N.s32_from_f32(x)
    xr = N.s32_to_f32(xs, cin)
    npad = ((n + bn - 1) // bn) * bn
    cw = N.ConvWeights(wt, bias, npad)
    out = N.s32_empty(b, h, w, (n + 31) // 32, DEV, zero=True)
    f32 = torch.zeros(b, n, h, w, device=DEV)
    N.conv_s32(N.S32Slice(xs), cw, bn, act="none", y0=N.S32Slice(out), f32=f32)
    torch.cuda.synchronize()
    ref, bound = _ref(xr, wt, bias, kh, kw)
    tol = 2e-6 * bound + 1e-6
    err = (f32.double() - ref).abs()
    assert bool((err <= tol).all()), f"fp32 out: max err {float(err.max()):.3e}, worst ratio {float((err / tol).max()):.2f}"
    got = N.s32_to_f32(out, n).double()
    err2 = (got - ref).abs()
    assert bool((err2 <= tol + 2.0 ** -22 * ref.abs()).all()), f"S32 out: max err {float(err2.max()):.3e}"
    # the plain PyTorch fp32 convolution of the original input on the GPU
    y32 = F.conv2d(x, wt, bias, padding=(kh // 2, kw // 2))
    rel = float((f32 - y32).abs().max() / y32.abs().max())
    assert rel <= 2e-6, rel


@pytest.mark.parametrize("kh,kw", [(1, 1), (3, 3), (1, 5), (5, 1)])
def test_conv_s32_integer_exact(kh, kw):
    """Small-integer operands: every product and partial sum is exact, so the result must be bit-exact."""
    g = torch.Generator().manual_seed(7 + kh * 10 + kw)
    b, cin, n, h, w = 2, 64, 128, 9, 36
    x = torch.randint(-8, 9, (b, cin, h, w), generator=g).float().to(DEV)
    wt = torch.randint(-4, 5, (n, cin, kh, kw), generator=g).float().to(DEV)
    wt[0] = 0
    wt[0, 0, kh // 2, kw // 2] = 1  # output channel 0 = input channel 0 (identity row)
    cw = N.ConvWeights(wt, None, 128)
    f32 = torch.empty(b, n, h, w, device=DEV)
    N.conv_s32(N.S32Slice(N.s32_from_f32(x)), cw, 128, f32=f32)
    ref = F.conv2d(x.double(), wt.double(), padding=(kh // 2, kw // 2))
    assert torch.equal(f32.double(), ref)
    assert torch.equal(f32[:, 0], x[:, 0])


def test_conv_s32_epilogues_slices_and_accumulate():
    g = torch.Generator().manual_seed(3)
    b, h, w = 2, 12, 40
    x = torch.randn(b, 256, h, w, generator=g).to(DEV)
    wt = (torch.randn(126, 256, 3, 3, generator=g) * 0.02).to(DEV)
    bias = torch.randn(126, generator=g).to(DEV)
    cw = N.ConvWeights(wt, bias, 128)
    xs = N.s32_from_f32(x)
    # destinations: channels 256..381 of two 12-group buffers; channels 382, 383 hold sentinels
    d0 = N.s32_from_f32(torch.full((b, 384, h, w), 7.0, device=DEV))
    d1 = d0.clone()
    N.conv_s32(N.S32Slice(xs), cw, 128, act="relu", out_scale=0.5, y0=N.S32Slice(d0, 8, 4), y1=N.S32Slice(d1, 8, 4))
    ref = _act(_ref(N.s32_to_f32(xs), wt, bias, 3, 3)[0], "relu") * 0.5
    for d in (d0, d1):
        got = N.s32_to_f32(d)
        assert float((got[:, 256:382].double() - ref).abs().max()) <= 1e-4
        assert bool((got[:, :256] == 7.0).all()) and bool((got[:, 382:] == 7.0).all())
    # fp32 accumulate into a (B, 2, H, W) tensor (flow head -> coords += delta)
    w2 = (torch.randn(2, 256, 3, 3, generator=g) * 0.02).to(DEV)
    cw2 = N.ConvWeights(w2, torch.tensor([0.5, -0.25], device=DEV), 32)
    coords = torch.randn(b, 2, h, w, device=DEV)
    c0 = coords.clone()
    N.conv_s32(N.S32Slice(xs), cw2, 32, f32=coords, f32_accumulate=True)
    delta = F.conv2d(N.s32_to_f32(xs).double(), w2.double(), cw2.bias.double(), padding=1)
    assert float((coords.double() - (c0.double() + delta)).abs().max()) <= 1e-5


@pytest.mark.parametrize("flags", [0, 256])
def test_conv_s32_gru_epilogues(flags):
    """z|r gates and the candidate/blend epilogue against the SepConvGRU math (update.py:91-97): the default gates
    (hardware exp2 / reciprocal, sigmoid_hw / tanh_hw) and, flags 256, libm's expf / tanhf; same bound."""
    lib = N.load()
    lib.oflow_exp_set_conv_flags(flags)
    try:
        _gru_epilogues()
    finally:
        lib.oflow_exp_set_conv_flags(0)


def _gru_epilogues():
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
    cq = N.ConvWeights(wq, bq, 128)
    z = torch.empty(b * h * w, ch, device=DEV)
    N.conv_s32(N.S32Slice(hx_s), czr, 128, epilogue=1, y0=N.S32Slice(rhx_s, 0, 4), gru_h=hmaster, gru_z=z)
    hxr = N.s32_to_f32(hx_s).double()
    zr_ref = torch.sigmoid(F.conv2d(hxr, wz.double(), bz.double(), padding=(0, 2)))
    r_ref = torch.sigmoid(F.conv2d(hxr, wr.double(), br.double(), padding=(0, 2)))
    zg = z.view(b, h, w, ch).permute(0, 3, 1, 2).double()
    assert float((zg - zr_ref).abs().max()) <= 2e-6
    rh_ref = r_ref * hx[:, :ch].double()
    rhx = N.s32_to_f32(rhx_s).double()
    assert float((rhx[:, :ch] - rh_ref).abs().max()) <= 2e-6
    assert torch.equal(rhx[:, ch:], hxr[:, ch:])
    h_ref = hx[:, :ch].double()
    N.conv_s32(N.S32Slice(rhx_s), cq, 128, epilogue=2, y0=N.S32Slice(hx_s, 0, 4), gru_h=hmaster, gru_z=z)
    q_ref = torch.tanh(F.conv2d(rhx, wq.double(), bq.double(), padding=(0, 2)))
    hn_ref = (1 - zg) * h_ref + zg * q_ref
    hn = hmaster.view(b, h, w, ch).permute(0, 3, 1, 2).double()
    assert float((hn - hn_ref).abs().max()) <= 2e-6
    assert float((N.s32_to_f32(hx_s)[:, :ch].double() - hn).abs().max()) <= 2.0 ** -21


@pytest.mark.parametrize("kh,kw", [(1, 5), (5, 1)])
def test_conv_s32_gru_hoisted_context(kh, kw):
    """The GRU with its loop-invariant context term hoisted (update.py:92-105, x = [inp | motion], inp constant):
    W_inp * inp + bias once (epilogue 0, fp32 NHWC [P, 384] = z | r | q), then the z|r and q convs over
    [h | motion | flow] only with that addend in their epilogues (oflow_conv_s32_ex3) -- against the full 384-channel
    SepConvGRU step in float64."""
    g = torch.Generator().manual_seed(17 + kh)
    b, h, w, ch = 2, 9, 37, 128
    full = torch.randn(b, 384, h, w, generator=g).to(DEV)
    full[:, :ch] = torch.tanh(full[:, :ch])
    full[:, ch : 2 * ch] = torch.relu(full[:, ch : 2 * ch])
    hmf = torch.cat([full[:, :ch], full[:, 2 * ch :]], dim=1)  # [h | motion | flow]
    hx_s = N.s32_from_f32(hmf)
    rhx_s = hx_s.clone()
    inp_s = N.s32_from_f32(full[:, ch : 2 * ch].contiguous())
    hmaster = full[:, :ch].permute(0, 2, 3, 1).reshape(-1, ch).contiguous()
    wz, wr, wq = ((torch.randn(ch, 384, kh, kw, generator=g) * 0.03).to(DEV) for _ in range(3))
    bz, br, bq = (torch.randn(ch, generator=g).to(DEV) for _ in range(3))
    sel = lambda wt: torch.cat([wt[:, :ch], wt[:, 2 * ch :]], dim=1)
    cinp = N.ConvWeights(torch.cat([wz, wr, wq])[:, ch : 2 * ch], torch.cat([bz, br, bq]), 384)
    czr = N.ConvWeights(sel(torch.cat([wz, wr])), None, 256)
    cq = N.ConvWeights(sel(wq), None, 128)
    gx = torch.empty(b * h * w, 384, device=DEV)
    N.conv_s32(N.S32Slice(inp_s), cinp, 128, nhwc=gx)
    z = torch.empty(b * h * w, ch, device=DEV)
    N.conv_s32(N.S32Slice(hx_s), czr, 128, epilogue=1, y0=N.S32Slice(rhx_s, 0, 4), gru_h=hmaster, gru_z=z,
               addend=gx[:, :256])
    # float64 reference on the exact operands (hi + lo of every S32 input)
    xr = torch.cat([N.s32_to_f32(hx_s)[:, :ch], N.s32_to_f32(inp_s), N.s32_to_f32(hx_s)[:, ch:]], dim=1).double()
    pad = (kh // 2, kw // 2)
    z_ref = torch.sigmoid(F.conv2d(xr, wz.double(), bz.double(), padding=pad))
    r_ref = torch.sigmoid(F.conv2d(xr, wr.double(), br.double(), padding=pad))
    zg = z.view(b, h, w, ch).permute(0, 3, 1, 2).double()
    assert float((zg - z_ref).abs().max()) <= 2e-6
    rhx = N.s32_to_f32(rhx_s).double()
    assert float((rhx[:, :ch] - r_ref * full[:, :ch].double()).abs().max()) <= 2e-6
    N.conv_s32(N.S32Slice(rhx_s), cq, 128, epilogue=2, y0=N.S32Slice(hx_s, 0, 4), gru_h=hmaster, gru_z=z,
               addend=gx[:, 256:])
    rxr = torch.cat([rhx[:, :ch], xr[:, ch:]], dim=1)
    q_ref = torch.tanh(F.conv2d(rxr, wq.double(), bq.double(), padding=pad))
    hn_ref = (1 - zg) * full[:, :ch].double() + zg * q_ref
    hn = hmaster.view(b, h, w, ch).permute(0, 3, 1, 2).double()
    assert float((hn - hn_ref).abs().max()) <= 2e-6
    # the addend is refused outside the GRU epilogues and with misaligned rows
    with pytest.raises(RuntimeError):
        N.conv_s32(N.S32Slice(hx_s), czr, 128, f32=torch.empty(b, 256, h, w, device=DEV), addend=gx[:, :256])
    with pytest.raises(RuntimeError):
        N.conv_s32(N.S32Slice(hx_s), czr, 128, epilogue=1, y0=N.S32Slice(rhx_s, 0, 4), gru_h=hmaster, gru_z=z,
                   addend=gx[:, 1:257])


def test_pack_s32_and_flow_prep():
    g = torch.Generator().manual_seed(5)
    b, h, w = 2, 11, 29
    cnet = torch.randn(b, 256, h, w, generator=g).to(DEV)
    hx = N.s32_empty(b, h, w, 12, DEV, zero=True)
    rhx = N.s32_empty(b, h, w, 12, DEV, zero=True)
    hm = torch.empty(b * h * w, 128, device=DEV)
    N.pack_s32(cnet[:, :128], "tanh", N.S32Slice(hx, 0, 4), nhwc=hm)
    N.pack_s32(cnet[:, 128:], "relu", N.S32Slice(hx, 4, 4), N.S32Slice(rhx, 4, 4))
    got = N.s32_to_f32(hx)
    assert float((got[:, :128] - torch.tanh(cnet[:, :128])).abs().max()) <= 1e-6
    assert torch.equal(hm.view(b, h, w, 128).permute(0, 3, 1, 2), torch.tanh(cnet[:, :128]))
    assert float((got[:, 128:256] - torch.relu(cnet[:, 128:])).abs().max()) <= 2e-6 * float(cnet.abs().max())
    assert torch.equal(N.s32_to_f32(rhx)[:, 128:256], got[:, 128:256])
    coords = coords_grid(b, h, w, device=DEV) + torch.randn(b, 2, h, w, generator=g).to(DEV) * 5
    pm = N.s32_empty(b, h, w, 4, DEV)
    N.flow_prep(coords, pm, (N.S32Slice(hx), 382), (N.S32Slice(rhx), 382))
    flow = coords - coords_grid(b, h, w, device=DEV)
    unf = F.unfold(flow, 7, padding=3).view(b, 2, 49, h, w).permute(0, 2, 1, 3, 4).reshape(b, 98, h, w)
    pmf = N.s32_to_f32(pm)
    assert float((pmf[:, :98] - unf).abs().max()) <= 1e-6 * float(flow.abs().max())
    assert bool((pmf[:, 98:] == 0).all())
    for t in (hx, rhx):
        assert float((N.s32_to_f32(t)[:, 382:] - flow).abs().max()) <= 1e-6 * float(flow.abs().max())


@pytest.mark.parametrize("b,h,w", [(4, 55, 128), (2, 11, 29), (1, 47, 156), (3, 5, 3)])
def test_convf1_from_flow_equals_patch_matrix(b, h, w):
    """convf1 straight from coords1 (N.FlowIn, OFLOW_IN_FLOW7: the flow window staged per tile, the patch operand built
    in LDS) against the conv of flow_prep's patch matrix: bit-identical S32 outputs (same patch values, same k order),
    ragged tiles and images smaller than a tile included; flow_prep without the matrix still writes the GRU inputs'
    flow channels bit for bit."""
    g = torch.Generator().manual_seed(h * 1000 + w)
    coords = coords_grid(b, h, w, device=DEV) + (torch.randn(b, 2, h, w, generator=g) * 9).to(DEV)
    conv = torch.nn.Conv2d(2, 128, 7, padding=3)
    with torch.no_grad():
        conv.weight.normal_(0.0, 0.05, generator=g)
        conv.bias.normal_(0.0, 0.1, generator=g)
    cw = N.ConvWeights(conv.weight.to(DEV), conv.bias.to(DEV), 128, patches=True)
    pm = N.s32_empty(b, h, w, 4, DEV, zero=True)
    hx = [N.s32_empty(b, h, w, 12, DEV, zero=True) for _ in range(2)]
    N.flow_prep(coords, pm, (N.S32Slice(hx[0]), 382))
    N.flow_prep(coords, None, (N.S32Slice(hx[1]), 382))
    ys = [N.s32_empty(b, h, w, 4, DEV, zero=True) for _ in range(2)]
    N.conv_s32(N.S32Slice(pm), cw, 128, "relu", y0=N.S32Slice(ys[0]))
    N.conv_s32(N.FlowIn(coords), cw, 128, "relu", y0=N.S32Slice(ys[1]))
    torch.cuda.synchronize()
    assert torch.equal(ys[0], ys[1])
    assert torch.equal(hx[0], hx[1])
    ref = F.relu(F.conv2d(coords.double() - coords_grid(b, h, w, device=DEV).double(), conv.weight.to(DEV).double(),
                          conv.bias.to(DEV).double(), padding=3))
    assert float((N.s32_to_f32(ys[1]).double() - ref).abs().max()) <= 1e-4 * max(1.0, float(ref.abs().max()))


@pytest.mark.parametrize("c,dst", [(100, 8), (37, 0), (256, 0), (8, 24)])
def test_pack_s32_ragged_channels(c, dst):
    """pack_s32 with channel counts that end mid-group / mid-octet and destinations that start mid-group: every
    destination value against the act'd source (hi + lo within fp32 rounding), the zero fill of the last octet, the
    neighbouring channels untouched, and the fp32 NHWC copy exact."""
    g = torch.Generator().manual_seed(c + dst)
    b, h, w = 2, 13, 37
    x = torch.randn(b, c, h, w, generator=g).to(DEV)
    groups = (dst + ((c + 7) // 8) * 8 + 31) // 32 + 1
    y = N.s32_from_f32(torch.full((b, groups * 32, h, w), 9.0, device=DEV))
    f = torch.empty(b * h * w, c, device=DEV)
    N.pack_s32(x, "relu", N.S32Slice(y), nhwc=f, dst_channel=dst)
    got = N.s32_to_f32(y).double()
    ref = torch.relu(x).double()
    assert float((got[:, dst : dst + c] - ref).abs().max()) <= 2.0 ** -21 * float(ref.abs().max())
    end = dst + ((c + 7) // 8) * 8
    assert bool((got[:, dst + c : end] == 0).all())
    assert bool((got[:, :dst] == 9.0).all()) and bool((got[:, end:] == 9.0).all())
    assert torch.equal(f.view(b, h, w, c).permute(0, 3, 1, 2), torch.relu(x))


@pytest.mark.parametrize("b,h,w", [(2, 11, 29), (4, 55, 128), (1, 47, 156), (3, 5, 3)])
def test_flow_prep_tiled_equals_per_thread(b, h, w):
    """The LDS-tiled flow_prep (default) against the per-thread form (experiment hook): patch matrix and the GRU inputs'
    flow channels bit-identical, ragged tiles and images smaller than a tile included."""
    g = torch.Generator().manual_seed(h * 100 + w)
    coords = coords_grid(b, h, w, device=DEV) + (torch.randn(b, 2, h, w, generator=g) * 7).to(DEV)
    lib = N.load()
    outs = []
    for untiled in (0, 1):
        lib.oflow_exp_set_flow_prep_untiled(untiled)
        try:
            pm = N.s32_empty(b, h, w, 4, DEV, zero=True)
            hx = N.s32_empty(b, h, w, 12, DEV, zero=True)
            rhx = N.s32_empty(b, h, w, 12, DEV, zero=True)
            N.flow_prep(coords, pm, (N.S32Slice(hx), 382), (N.S32Slice(rhx), 382))
            torch.cuda.synchronize()
            outs.append((pm, hx, rhx))
        finally:
            lib.oflow_exp_set_flow_prep_untiled(0)
    for u, v in zip(*outs):
        assert torch.equal(u, v)


@pytest.mark.parametrize("c,n,bn", [(64, 64, 64), (96, 96, 96), (128, 128, 128)])
def test_conv_normalise_on_load_equals_norm_apply(c, n, bn):
    """oflow_conv_s32_ex2 with a raw fp32 NHWC input normalised + ReLU'd while staged (NhwcNormIn) equals the
    two-pass path: norm_apply -> S32 -> conv (extractor.py:75-76 between a block's two convs)."""
    b, h, w = 2, 37, 70
    g = torch.Generator().manual_seed(5)
    raw = (torch.randn(b * h * w, c, generator=g) * 3 + 0.5).to(DEV)
    alpha = (torch.rand(b, c, generator=g) + 0.5).to(DEV)
    beta = torch.randn(b, c, generator=g).to(DEV)
    wt = (torch.randn(n, c, 3, 3, generator=g) * 0.05).to(DEV)
    cw = N.ConvWeights(wt, torch.randn(n, generator=g).to(DEV) * 0.1, ((n + 31) // 32) * 32)
    s32 = N.s32_empty(b, h, w, c // 32, DEV)
    N.norm_apply(raw, (b, c, h, w), alpha, beta, "relu", N.S32Slice(s32))
    y1 = torch.zeros(b, n, h, w, device=DEV)
    y2 = torch.zeros(b, n, h, w, device=DEV)
    N.conv_s32(N.S32Slice(s32), cw, bn, f32=y1)
    N.conv_s32(N.NhwcNormIn(raw, b, h, w, alpha, beta), cw, bn, f32=y2)
    torch.cuda.synchronize()
    err = float((y1 - y2).abs().max())
    assert err <= 1e-6 * float(y1.abs().max()), err


@pytest.mark.parametrize("sigma", [0.0, 3.0, 25.0])
@pytest.mark.parametrize("radius,levels", [(4, 4), (2, 3), (3, 5), (7, 2)])
@pytest.mark.parametrize("pad", [0, 12])
def test_lookup_nhwc_equals_lookup(sigma, radius, levels, pad):
    """oflow_corr_lookup_tiled_nhwc_f32 (the RAFT forward's lookup: segment-DMA gathers, query-major waves) = the
    NCHW lookup permuted to NHWC, bit for bit; row pitch = L*K*K (dense, float4 stores) or padded (scalar stores, the
    pad channels untouched); ragged last wave (33*37*2 queries)."""
    g = torch.Generator().manual_seed(int(sigma) + 7 * radius)
    b, c, h, w = 2, 256, 33, 37
    f1 = torch.randn(b, c, h, w, generator=g).to(DEV)
    f2 = torch.randn(b, c, h, w, generator=g).to(DEV)
    pyr = N.corr_pyramid_tiled(f1, f2, levels)
    coords = coords_grid(b, h, w, device=DEV) + torch.randn(b, 2, h, w, generator=g).to(DEV) * sigma
    ref = N.corr_lookup_tiled(pyr, coords, radius)  # (B, L*K*K, H, W)
    ch = levels * (2 * radius + 1) ** 2
    out = torch.full((b * h * w, ch + pad), 7.0, device=DEV)
    N.corr_lookup_tiled_nhwc(pyr, coords, radius, out)
    got = out.view(b, h, w, ch + pad)
    assert torch.equal(got[..., :ch], ref.permute(0, 2, 3, 1))
    assert bool((got[..., ch:] == 7.0).all())


@pytest.mark.parametrize("c", [352, 324, 100])
def test_conv_f32_input_equals_s32_input(c):
    """convc1 reading fp32 NHWC rows (F32In, split while staged; rows of C floats, channels past C staged as zeros,
    C = 324 is the lookup row) = reading the same values as S32."""
    g = torch.Generator().manual_seed(3)
    b, h, w, n = 2, 23, 45, 256
    x = (torch.randn(b * h * w, c, generator=g) * 4).to(DEV)
    s32 = N.s32_from_f32(x.view(b, h, w, c).permute(0, 3, 1, 2).contiguous())
    wt = (torch.randn(n, c, 1, 1, generator=g) * 0.05).to(DEV)
    cw = N.ConvWeights(wt, torch.randn(n, generator=g).to(DEV) * 0.1, 256)
    y1 = N.s32_empty(b, h, w, 8, DEV, zero=True)
    y2 = N.s32_empty(b, h, w, 8, DEV, zero=True)
    N.conv_s32(N.S32Slice(s32), cw, 128, "relu", y0=N.S32Slice(y1))
    N.conv_s32(N.F32In(x, b, h, w), cw, 128, "relu", y0=N.S32Slice(y2))
    torch.cuda.synchronize()
    assert torch.equal(y1, y2)


@pytest.mark.parametrize("b,c,h,w", [(2, 3, 40, 70), (1, 3, 9, 131), (1, 1, 16, 16)])
def test_stem_patches_match_unfold(b, c, h, w):
    """oflow_stem_patches_s32 (LDS-staged 7x7/2 pad-3 patch matrix, channel t*C + c) = F.unfold of the image, as
    hi + lo (exact for these small integers), zeros past 49*C; ragged last workgroup (Wo % 64 != 0)."""
    g = torch.Generator().manual_seed(b * 100 + w)
    img = torch.randint(0, 256, (b, c, h, w), generator=g).float().to(DEV)
    groups = (49 * c + 31) // 32
    out = N.s32_empty(b, (h + 1) // 2, (w + 1) // 2, groups, DEV)
    N.stem_patches(img, out)
    got = N.s32_to_f32(out)  # (B, G*32, Ho, Wo)
    ho, wo = (h + 1) // 2, (w + 1) // 2
    unf = F.unfold(img, 7, padding=3, stride=2).view(b, c, 49, ho, wo)  # channel c*49 + t
    ref = unf.permute(0, 2, 1, 3, 4).reshape(b, 49 * c, ho, wo)  # -> t*C + c
    assert torch.equal(got[:, : 49 * c], ref)
    assert bool((got[:, 49 * c :] == 0).all())


def test_range_check_fires_on_fp16_overflow(monkeypatch):
    """OFLOW_CHECK=1 (here: the module flag it sets): a convolution input outside the fp16 range of the split operands
    raises -- an S32 input whose hi half overflowed to inf, an fp32 input staged by the kernel, a normalise-on-load
    input -- while in-range inputs pass."""
    monkeypatch.setattr(N, "CHECK_RANGE", True)
    g = torch.Generator().manual_seed(5)
    b, c, h, w = 1, 64, 8, 12
    x = torch.randn(b, c, h, w, generator=g).to(DEV)
    cw = N.ConvWeights((torch.randn(32, c, 1, 1, generator=g) * 0.1).to(DEV), None, 32)
    out = torch.empty(b, 32, h, w, device=DEV)
    N.conv_s32(N.S32Slice(N.s32_from_f32(x)), cw, 32, f32=out)  # in range: runs
    big = x.clone()
    big[0, 5, 3, 4] = 7.0e4
    with pytest.raises(RuntimeError, match="fp16 range"):
        N.conv_s32(N.S32Slice(N.s32_from_f32(big)), cw, 32, f32=out)
    rows = big.permute(0, 2, 3, 1).reshape(b * h * w, c).contiguous()
    with pytest.raises(RuntimeError, match="fp16 range"):
        N.conv_s32(N.F32In(rows, b, h, w), cw, 32, f32=out)
    cw3 = N.ConvWeights((torch.randn(32, c, 3, 3, generator=g) * 0.1).to(DEV), None, 32)
    scale = torch.ones(b, c, device=DEV)
    shift = torch.zeros(b, c, device=DEV)
    shift[0, 9] = 1.0e5
    with pytest.raises(RuntimeError, match="fp16 range"):
        N.conv_s32(N.NhwcNormIn(rows.clamp(-10, 10), b, h, w, scale, shift), cw3, 32, f32=out)
    monkeypatch.setattr(N, "CHECK_RANGE", False)
    N.conv_s32(N.S32Slice(N.s32_from_f32(big)), cw, 32, f32=out)  # off: no check, no raise


@pytest.mark.parametrize("tiled", [False, True])
@pytest.mark.parametrize("b,h,w", [(2, 55, 128), (1, 7, 9), (3, 16, 33), (4, 55, 128)])
def test_flow_head2_matches_fp64(b, h, w, tiled):
    """The flow head's 2-channel output conv as fp32 FMAs (oflow_flow_head2_s32, and the LDS-tiled large-grid form
    oflow_flow_head2_tiled_s32) added into coords, vs float64; the small grids put most pixels on the zero-padded
    border, ragged tiles included."""
    g = torch.Generator().manual_seed(h * w)
    x = (torch.randn(b, 256, h, w, generator=g) * 1.5).to(DEV)
    wt = (torch.randn(2, 256, 3, 3, generator=g) / 48.0).to(DEV)
    bias = torch.randn(2, generator=g).to(DEV)
    xs = N.s32_from_f32(x)
    xr = N.s32_to_f32(xs, 256)
    coords = torch.randn(b, 2, h, w, generator=g).to(DEV)
    ref = coords.double() + F.conv2d(xr.double(), wt.double(), bias.double(), padding=1)
    bound = F.conv2d(xr.double().abs(), wt.double().abs(), None, padding=1)
    if tiled:
        N.flow_head2_tiled(N.S32Slice(xs), N.flow_head2_tiled_weights(wt), bias, coords)
    else:
        N.flow_head2(N.S32Slice(xs), wt.contiguous(), bias, coords)
    torch.cuda.synchronize()
    err = (coords.double() - ref).abs()
    tol = 2e-6 * bound + 1e-6 + 2.0 ** -23 * ref.abs()
    assert bool((err <= tol).all()), float(err.max())


def test_flow_head2_arg_errors():
    xs = N.s32_empty(1, 8, 8, 8, DEV)
    coords = torch.zeros(1, 2, 8, 8, device=DEV)
    conv = torch.nn.Conv2d(256, 2, 3, padding=1).to(DEV)
    wt, bias = conv.weight.detach().contiguous(), conv.bias.detach()
    with pytest.raises(RuntimeError):
        N.flow_head2(N.S32Slice(xs), wt[:, :128].contiguous(), bias, coords)  # channel count must match the slice
    with pytest.raises(RuntimeError):
        N.flow_head2(N.S32Slice(xs), wt, None, coords)  # bias required
    with pytest.raises(RuntimeError):
        N.flow_head2(N.S32Slice(xs), wt, bias, coords[:, :, :4])


@pytest.mark.parametrize("kh,c,n,bn,h,w,tiles8", [(3, 64, 64, 64, 37, 70, 0), (3, 64, 64, 64, 37, 70, 1),
                                                   (3, 96, 96, 96, 21, 40, 0), (3, 128, 128, 128, 13, 33, 0),
                                                   (1, 64, 96, 96, 16, 64, 0), (2, 256, 128, 128, 11, 20, 0)])
def test_instance_norm_partials(kh, c, n, bn, h, w, tiles8):
    """The conv epilogue's per-tile instance-norm partials (count, mean, M2 from the accumulators: per lane, lane
    halves, then the waves of each 4-row sub-tile) merged by oflow_norm_stats_finalize = the per-(image, channel)
    mean / variance of the conv's own fp32 output computed in float64 (extractor.py:75-76, nn.InstanceNorm2d eps 1e-5):
    alpha = 1/sqrt(var + eps) and beta = -mean * alpha to 2e-6 relative (fp32 partial sums over <= 128 pixels); ragged
    H and W (partial tiles), 4-row and 8-row tiles (oflow_exp_set_stats_8row), 64 / 96 / 128-channel blocks."""
    import ctypes
    b = 2
    g = torch.Generator().manual_seed(11 + kh + n + tiles8)
    x = (torch.randn(b, c, h, w, generator=g) * 2 + 0.3).to(DEV)
    wt = (torch.randn(n, c, kh, kh, generator=g) * 0.05).to(DEV)
    cw = N.ConvWeights(wt, torch.randn(n, generator=g).to(DEV) * 0.5, ((n + 31) // 32) * 32)
    tiles = N.conv_tiles(h, w)
    raw = torch.empty(b * h * w, n, device=DEV)
    part = torch.full((b, tiles, cw.n_pad, 3), float("nan"), device=DEV)
    lib = N.load()
    lib.oflow_exp_set_stats_8row.argtypes = [ctypes.c_int]
    lib.oflow_exp_set_stats_8row(tiles8)
    try:
        N.conv_s32(N.S32Slice(N.s32_from_f32(x)), cw, bn, nhwc=raw, stats=part)
        alpha, beta = N.norm_stats(part, b, tiles, cw.n_pad, n, 1e-5)
        torch.cuda.synchronize()
    finally:
        lib.oflow_exp_set_stats_8row(0)
    y = raw.view(b, h * w, n).double()
    mean = y.mean(dim=1)
    var = y.var(dim=1, unbiased=False)
    a_ref = 1.0 / torch.sqrt(var + 1e-5)
    b_ref = -mean * a_ref
    assert torch.isfinite(part[..., :n, :]).all()
    ea = float(((alpha.double() - a_ref).abs() / a_ref).max())
    eb = float(((beta.double() - b_ref).abs() / (mean.abs() * a_ref + 1.0)).max())
    assert ea <= 2e-6 and eb <= 2e-6, (ea, eb)


@pytest.mark.parametrize("b,h,w", [(4, 55, 128), (2, 13, 45), (1, 1, 1), (3, 47, 156)])
def test_flow_head_col2im_matches_fp64_and_conv(b, h, w):
    """The flow head's output conv (update.py:36, 3x3 256 -> 2, bias; raft.py:133 coords1 += delta) as a 1x1 conv
    256 -> 18 (per-tap products) + oflow_flow_head_col2im_f32, against float64 F.conv2d of the same split operands, and
    against the 3x3 conv_s32 path (fp32 reordering apart): borders (zero padding), a 1x1 grid, KITTI's 47x156."""
    from model.update import SplitUpdate  # noqa: F401  (the weight layout under test is SplitUpdate's "fh2T")

    g = torch.Generator().manual_seed(b * 1000 + h + w)
    x = torch.relu(torch.randn(b, 256, h, w, generator=g) * 2.0).to(DEV)
    wt = (torch.randn(2, 256, 3, 3, generator=g) / math.sqrt(256 * 9)).to(DEV)
    bias = torch.randn(2, generator=g).to(DEV)
    coords = (torch.randn(b, 2, h, w, generator=g) * 30.0).to(DEV)
    xs = N.s32_from_f32(x)
    xe = N.s32_to_f32(xs, 256)  # the exact operand values the kernels see (hi + lo)
    ref, bound = _ref(xe, wt, bias, 3, 3)
    ref = ref + coords.double()
    cw_t = N.ConvWeights(wt.permute(2, 3, 0, 1).reshape(18, 256, 1, 1), None, 32)
    y = torch.empty(b, 18, h, w, device=DEV)
    c1 = coords.clone()
    with torch.inference_mode():
        N.conv_s32(N.S32Slice(xs), cw_t, 32, f32=y)
        N.flow_head_col2im(y, bias, c1)
        c2 = coords.clone()
        N.conv_s32(N.S32Slice(xs), N.ConvWeights(wt, bias, 32), 32, f32=c2, f32_accumulate=True)
    tol = 2e-6 * bound + 1e-6 + 2e-7 * coords.double().abs()
    assert bool(((c1.double() - ref).abs() <= tol).all()), float((c1.double() - ref).abs().max())
    assert bool(((c2.double() - ref).abs() <= tol).all())
    assert float((c1 - c2).abs().max()) <= 1e-4


@pytest.mark.parametrize("kh,kw,cin,n,bn,epi,stats,b,h,w", [
    (3, 3, 256, 128, 128, 0, False, 2, 70, 130),   # even group count
    (3, 3, 352, 128, 128, 0, False, 1, 131, 131),  # odd group count with odd taps: the two-group body's one-group tail
    (3, 3, 32, 128, 128, 0, False, 4, 45, 97),     # one group
    (1, 5, 384, 256, 128, 1, False, 2, 66, 130),   # GRU z|r gates (epilogue 1)
    (5, 1, 384, 128, 128, 2, False, 2, 66, 130),   # GRU candidate (epilogue 2)
    (5, 1, 96, 128, 128, 0, False, 3, 61, 100),    # odd group count, odd taps
    (3, 3, 128, 128, 128, 0, True, 2, 27, 64),     # with instance-norm partials: the LDS-staged kernel (wf ignored)
    (3, 3, 256, 192, 64, 0, False, 2, 55, 128),    # convc2's shape, 64-channel blocks (CONV_BREG64: 2 x 2 waves)
    (3, 3, 96, 64, 64, 0, False, 3, 41, 133),      # 64-channel blocks, odd group count, ragged tiles
    (3, 3, 256, 2, 32, 0, False, 2, 55, 128),      # the flow head's output conv (CONV_BREG32: 4 x 1 waves)
])
def test_conv_register_weights_bit_identical(monkeypatch, kh, kw, cin, n, bn, epi, stats, b, h, w):
    """The register-direct weight path (ConvWeights.frag -> oflow_conv_s32_ex4, BREG kernels; grids over 16384 output
    pixels at block_n 128, no instance-norm partials) against the LDS-staged one: the same MFMAs in the same order per
    output, so every output bit-identical; plus the fp64 bound of test_conv_s32_matches_fp64 for the plain epilogue."""
    g = torch.Generator().manual_seed(kh * 100 + cin + epi + n)
    x = (torch.randn(b, cin, h, w, generator=g) * 1.5).to(DEV)
    wt = (torch.randn(n, cin, kh, kw, generator=g) / math.sqrt(cin * kh * kw)).to(DEV)
    bias = torch.randn(n, generator=g).to(DEV)
    npad = -(-n // bn) * bn
    cw = N.ConvWeights(wt, bias, npad)
    xs = N.s32_from_f32(x)
    ch = 128

    def run(breg):
        monkeypatch.setattr(N, "CONV_BREG", breg)
        monkeypatch.setattr(N, "CONV_BREG64", breg)
        monkeypatch.setattr(N, "CONV_BREG32", breg)
        y = N.s32_empty(b, h, w, -(-n // 32) if epi == 0 else 4, DEV, zero=True)
        if stats:
            raw = torch.zeros(b * h * w, n, device=DEV)
            part = torch.zeros(b, N.conv_tiles(h, w), npad, 3, device=DEV)
            N.conv_s32(N.S32Slice(xs), cw, bn, nhwc=raw, stats=part)
            torch.cuda.synchronize()
            return raw, part, None, None
        if epi == 0:
            f32 = torch.zeros(b, n, h, w, device=DEV)
            N.conv_s32(N.S32Slice(xs), cw, bn, act="relu", y0=N.S32Slice(y), f32=f32)
            torch.cuda.synchronize()
            return f32, y, None, None
        hm = torch.tanh(torch.randn(b * h * w, ch, generator=torch.Generator().manual_seed(1))).to(DEV)
        z = torch.rand(b * h * w, ch, generator=torch.Generator().manual_seed(2)).to(DEV)
        N.conv_s32(N.S32Slice(xs), cw, bn, epilogue=epi, y0=N.S32Slice(y), gru_h=hm, gru_z=z)
        torch.cuda.synchronize()
        return None, y, hm, z

    a, c = run(True), run(False)
    for u, v in zip(a, c):
        if u is not None:
            assert torch.equal(u, v)
    if epi == 0 and not stats:
        ref, bound = _ref(N.s32_to_f32(xs, cin), wt, bias, kh, kw)
        err = (a[0].double() - torch.relu(ref)).abs()
        assert bool((err <= 2e-6 * bound + 1e-6).all()), float(err.max())


