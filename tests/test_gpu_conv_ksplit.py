"""Split-K register-direct convolutions (oflow_conv_s32_ex5, include/oflow.h; csrc/conv_s32.hip): each 4 x 32-pixel
tile runs as two workgroups over half the input groups each, meeting through an fp32 slab and agent-scope counters.
The RAFT update uses it for the motion conv and both GRU candidate convs (update.py:91-128; model/update.py
KSPLIT_LAYERS). Checked against a float64 conv of the same split operands (the conv_s32 bound), against the unsplit
kernel, exactly on small integers, across repeated calls sharing one scratch (counters that only grow), on two
streams at once. The RAFT forward leaves it off by default (model/update.py KSPLIT_LAYERS: slower in the two-lane step);
test_raft_with_ksplit_matches_reference_flows runs the benchmarked forward with it on against the reference's flows."""
import math

import pytest
import torch
import torch.nn.functional as F

from optical_flow import _native as N

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


CASES = [
    # kh, kw, cin, n, block_n, B, H, W
    (3, 3, 256, 126, 128, 4, 55, 128),  # the motion conv of a 4-pair Sintel lane (224 tiles)
    (1, 5, 256, 128, 128, 4, 55, 128),  # the GRU candidate convs' shapes
    (5, 1, 256, 128, 128, 2, 47, 156),  # KITTI grid: ragged tiles in x and y
    (3, 3, 256, 126, 128, 1, 13, 45),   # a small grid: split calls keep the default tiles
    (3, 3, 384, 128, 128, 2, 20, 64),   # 12 input groups (6 per workgroup)
    (3, 3, 64, 256, 128, 2, 6, 33),     # two channel blocks per tile (n_pad 256)
]


@pytest.mark.parametrize("kh,kw,cin,n,bn,b,h,w", CASES)
def test_ksplit_matches_fp64_and_unsplit(kh, kw, cin, n, bn, b, h, w):
    g = torch.Generator().manual_seed(kh * 100 + kw * 10 + cin + n + h)
    x = (torch.randn(b, cin, h, w, generator=g) * 1.5).to(DEV)
    wt = (torch.randn(n, cin, kh, kw, generator=g) / math.sqrt(cin * kh * kw)).to(DEV)
    bias = torch.randn(n, generator=g).to(DEV)
    xs = N.s32_from_f32(x)
    npad = ((n + bn - 1) // bn) * bn
    cw = N.ConvWeights(wt, bias, npad)
    ks = N.KSplit(b, h, w, DEV, block_n=bn, blocks=npad // bn)
    f_split = torch.zeros(b, n, h, w, device=DEV)
    f_plain = torch.zeros(b, n, h, w, device=DEV)
    out = N.s32_empty(b, h, w, (n + 31) // 32, DEV, zero=True)
    N.conv_s32(N.S32Slice(xs), cw, bn, f32=f_split, y0=N.S32Slice(out), ksplit=ks)
    N.conv_s32(N.S32Slice(xs), cw, bn, f32=f_plain)
    torch.cuda.synchronize()
    ref, bound = _ref(N.s32_to_f32(xs, cin), wt, bias, kh, kw)
    tol = 2e-6 * bound + 1e-6
    err = (f_split.double() - ref).abs()
    assert bool((err <= tol).all()), f"split: max err {float(err.max()):.3e}, worst ratio {float((err / tol).max()):.2f}"
    got = N.s32_to_f32(out, n).double()
    assert bool(((got - ref).abs() <= tol + 2.0 ** -22 * ref.abs()).all())
    # split vs unsplit: one more fp32 addition per output, same bound
    assert bool(((f_split.double() - f_plain.double()).abs() <= 2e-6 * bound + 1e-6).all())
    # counters: two tickets and one publication per tile of this call
    tiles = b * N.conv_tiles(h, w) * (npad // bn)
    ctr = ks.ctr.view(-1, 2)[:tiles].cpu()
    assert bool((ctr[:, 0] == 2).all()) and bool((ctr[:, 1] == 1).all())


@pytest.mark.parametrize("kh,kw", [(3, 3), (1, 5), (5, 1)])
def test_ksplit_integer_exact(kh, kw):
    """Small-integer operands: every partial sum is exact in fp32, so the split result is the exact result."""
    g = torch.Generator().manual_seed(31 + kh * 10 + kw)
    b, cin, n, h, w = 2, 256, 128, 11, 70
    x = torch.randint(-8, 9, (b, cin, h, w), generator=g).float().to(DEV)
    wt = torch.randint(-4, 5, (n, cin, kh, kw), generator=g).float().to(DEV)
    cw = N.ConvWeights(wt, None, 128)
    f32 = torch.empty(b, n, h, w, device=DEV)
    N.conv_s32(N.S32Slice(N.s32_from_f32(x)), cw, 128, f32=f32, ksplit=N.KSplit(b, h, w, DEV))
    ref = F.conv2d(x.double(), wt.double(), padding=(kh // 2, kw // 2))
    assert torch.equal(f32.double(), ref)


def test_ksplit_repeated_calls_and_two_streams():
    """One scratch reused by many stream-ordered calls (the counters keep growing: no reset) gives the same bits every
    time; two streams with their own scratch run concurrently and give the same bits too."""
    g = torch.Generator().manual_seed(5)
    b, h, w = 4, 55, 128
    x = (torch.randn(b, 256, h, w, generator=g)).to(DEV)
    wt = (torch.randn(126, 256, 3, 3, generator=g) * 0.02).to(DEV)
    cw = N.ConvWeights(wt, torch.randn(126, generator=g).to(DEV), 128)
    xs = N.s32_from_f32(x)
    ks = N.KSplit(b, h, w, DEV)
    first = torch.empty(b, 126, h, w, device=DEV)
    N.conv_s32(N.S32Slice(xs), cw, 128, act="relu", f32=first, ksplit=ks)
    outs = []
    for _ in range(7):
        o = torch.empty_like(first)
        N.conv_s32(N.S32Slice(xs), cw, 128, act="relu", f32=o, ksplit=ks)
        outs.append(o)
    torch.cuda.synchronize()
    assert all(torch.equal(o, first) for o in outs)
    tiles = b * N.conv_tiles(h, w)
    ctr = ks.ctr.view(-1, 2)[:tiles].cpu()
    assert bool((ctr[:, 0] == 16).all()) and bool((ctr[:, 1] == 8).all())
    streams = [torch.cuda.Stream(device=DEV) for _ in range(2)]
    scratch = [N.KSplit(b, h, w, DEV) for _ in range(2)]
    res = [[], []]
    cur = torch.cuda.current_stream(DEV)
    for st in streams:
        st.wait_stream(cur)
    for _ in range(4):
        for i, st in enumerate(streams):
            with torch.cuda.stream(st):
                o = torch.empty_like(first)
                N.conv_s32(N.S32Slice(xs), cw, 128, act="relu", f32=o, ksplit=scratch[i])
                res[i].append(o)
    for st in streams:
        cur.wait_stream(st)
    torch.cuda.synchronize()
    assert all(torch.equal(o, first) for r in res for o in r)


@pytest.mark.parametrize("kh,kw", [(1, 5), (5, 1)])
def test_ksplit_gru_candidate_epilogue(kh, kw):
    """The GRU candidate + blend epilogue (update.py:96-97) after a split main loop: h = (1 - z) h + z tanh(q + addend)
    against float64, and against the unsplit kernel."""
    g = torch.Generator().manual_seed(41 + kh)
    b, h, w, ch = 4, 55, 128, 128
    rhx = torch.randn(b, 256, h, w, generator=g).to(DEV)
    rhx_s = N.s32_from_f32(rhx)
    wq = (torch.randn(ch, 256, kh, kw, generator=g) * 0.03).to(DEV)
    cq = N.ConvWeights(wq, None, 128)
    z = torch.rand(b * h * w, ch, generator=g).to(DEV)
    h0 = torch.tanh(torch.randn(b * h * w, ch, generator=g)).to(DEV)
    gx = torch.randn(b * h * w, ch, generator=g).to(DEV)
    res = {}
    for split in (False, True):
        hm = h0.clone()
        hx_s = N.s32_empty(b, h, w, 4, DEV, zero=True)
        N.conv_s32(N.S32Slice(rhx_s), cq, 128, epilogue=2, y0=N.S32Slice(hx_s), gru_h=hm, gru_z=z, addend=gx,
                   ksplit=N.KSplit(b, h, w, DEV) if split else None)
        res[split] = hm
    torch.cuda.synchronize()
    q, bound = _ref(N.s32_to_f32(rhx_s), wq, None, kh, kw)
    q = torch.tanh(q.permute(0, 2, 3, 1).reshape(-1, ch) + gx.double())
    bound = bound.permute(0, 2, 3, 1).reshape(-1, ch)
    ref = (1 - z.double()) * h0.double() + z.double() * q
    # the conv_s32 bound on the pre-activation, through tanh (slope <= 1) and the z-weighted blend, + blend rounding
    tol = z.double() * (2e-6 * bound + 1e-6) + 2.0 ** -22
    for split in (True, False):
        err = (res[split].double() - ref).abs()
        assert bool((err <= tol).all()), (split, float(err.max()), float((err / tol).max()))
    assert bool(((res[True] - res[False]).abs().double() <= 2 * tol).all())


def test_ksplit_arg_errors():
    b, h, w = 2, 9, 40
    x = N.s32_from_f32(torch.randn(b, 256, h, w, device=DEV))
    cw = N.ConvWeights(torch.randn(128, 256, 3, 3, device=DEV) * 0.02, None, 128)
    small = N.KSplit(1, h, w, DEV)  # one image's tiles: too small for two
    with pytest.raises(RuntimeError):
        N.conv_s32(N.S32Slice(x), cw, 128, f32=torch.empty(b, 128, h, w, device=DEV), ksplit=small)
    lib = N.load()
    f = torch.empty(b, 128, h, w, device=DEV)
    ks = N.KSplit(b, h, w, DEV)
    xv = N.S32Slice(x)
    args = [xv.ptr, xv.ps, 8, cw.pack.data_ptr(), 128, cw.wscale.data_ptr(), None, 128, b, h, w, 3, 3, 128,
            0, 0, 1.0, None, 0, None, 0, f.data_ptr(), f.stride(0), f.stride(1), 0, None, None, 0, None, 0, None, None, 0,
            0, 0, 0, None, None, None, 0, cw.frag().data_ptr()]
    stream = torch.cuda.current_stream(DEV).cuda_stream
    assert lib.oflow_conv_s32_ex5(*args, ks.slab.data_ptr(), None, ks.tiles, stream) == -1  # OFLOW_E_NULL
    assert lib.oflow_conv_s32_ex5(*args, ks.slab.data_ptr() + 4, ks.ctr.data_ptr(), ks.tiles, stream) == -7  # OFLOW_E_ALIGN
    assert lib.oflow_conv_s32_ex5(*args, ks.slab.data_ptr(), ks.ctr.data_ptr(), 0, stream) == -2  # OFLOW_E_SHAPE
    assert lib.oflow_conv_s32_ex5(*args, ks.slab.data_ptr(), ks.ctr.data_ptr(), ks.tiles, stream) == 0
    torch.cuda.synchronize()


def test_raft_with_ksplit_matches_reference_flows():
    """The benchmarked forward (8 Sintel pairs, two lanes, 12 iterations) with the motion conv and the GRU candidate
    convs split: the reference's flows for those pairs at the SURVEY §8(c) bar, and single lane = two lanes bit for bit."""
    import os

    import numpy as np

    from model import RAFT, InputPadder, synthetic
    from model import update as U

    g = np.load(os.path.join(os.path.dirname(__file__), "golden", "raft_e2e_batch.npz"), allow_pickle=False)
    b, h, w, iters, _, seed = (int(v) for v in g["sintel8_cfg"])
    img0, img1 = synthetic.synthetic_pair(b, h, w, seed=seed)
    padder = InputPadder(img0.shape, mode=str(g["sintel8_mode"]))
    model = RAFT().eval()
    model.load_state_dict(synthetic.synthetic_state_dict(model.state_dict()))
    model = model.to(DEV)
    saved = U.KSPLIT_LAYERS
    U.KSPLIT_LAYERS = frozenset({"mo", "q"})
    try:
        with torch.inference_mode():
            p0, p1 = padder.pad(img0.to(DEV), img1.to(DEV))
            outs = {}
            for lanes in (2, 1):
                model.pair_lanes = lanes
                outs[lanes] = model(p0, p1, iters=iters, test_mode=True)
    finally:
        U.KSPLIT_LAYERS = saved
    assert torch.equal(outs[1][0], outs[2][0]) and torch.equal(outs[1][1], outs[2][1])
    low = outs[2][0].cpu()
    epe = torch.norm(low - torch.from_numpy(g["sintel8_low"]), dim=1)
    assert float(epe.mean()) <= 1e-4 and float(epe.max()) <= 1e-3, (float(epe.mean()), float(epe.max()))
