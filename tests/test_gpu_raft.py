"""End-to-end RAFT inference on the GPU (product model: HIP corr/lookup + MIOpen convs) against the flows the
reference itself produced on CPU (tests/golden/raft_e2e.npz), with hash weights and synthetic frames.

Tolerance: mean EPE <= 1e-4 px and max EPE <= 1e-3 px on the low-res flow and on the
upsampled flow. To separate our kernels from the convolution backend, the same forward is also run with the
oracle's PyTorch correlation ops on the GPU ("oracle-on-GPU"); the product must agree with it far tighter than
with the CPU goldens if a deviation came from MIOpen's convolutions rather than from the HIP kernels.
"""
import numpy as np
import pytest
import torch

from model import RAFT, InputPadder, synthetic
from oracle import raft as oraft

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)


def _model(cls):
    m = cls().eval()
    m.load_state_dict(synthetic.synthetic_state_dict(m.state_dict()))
    return m.to(DEV)


def _epe(a, b):
    e = torch.norm(a.float().cpu() - torch.as_tensor(b), p=2, dim=1)
    return float(e.mean()), float(e.max())


@pytest.mark.parametrize("impl", ["split", "fused", "split+module-encoders"])
@pytest.mark.parametrize("tag", ["small", "small24", "kittimode", "sintel", "kitti"])
def test_raft_matches_reference_flows(golden, tag, impl):
    g = golden("raft_e2e")
    b, h, w, iters, s, seed = (int(v) for v in g[f"{tag}_cfg"])
    img0, img1 = synthetic.synthetic_pair(b, h, w, seed=seed)
    padder = InputPadder(img0.shape, mode=str(g[f"{tag}_mode"]))
    p0, p1 = (x.to(DEV) for x in padder.pad(img0, img1))
    model = _model(RAFT)
    model.update_impl = impl.split("+")[0]
    if impl.endswith("module-encoders") or impl == "fused":
        model.encoder_impl = "module"
    with torch.inference_mode():
        low, up = model(p0, p1, iters=iters, test_mode=True)
    up = padder.unpad(up)[..., ::s, ::s]
    ml, xl = _epe(low, g[f"{tag}_low"])
    mu, xu = _epe(up, g[f"{tag}_up"])
    print(f"{tag} [{impl}]: low EPE mean {ml:.2e} max {xl:.2e}; up EPE mean {mu:.2e} max {xu:.2e}")
    assert ml <= 1e-4 and mu <= 1e-4, (ml, mu)
    assert xl <= 1e-3 and xu <= 1e-3, (xl, xu)


@pytest.mark.parametrize("tag", ["sintel8", "kitti8"])
def test_raft_matches_reference_flows_at_benchmarked_batch(golden, tag):
    """The forward bench.py times (8 pairs per GPU, 12 iterations, 'sintel' padding, default model: split encoders,
    split-fp16 pyramid, lookup fused into convc1, two pair lanes, the flow head's output conv on the tiled fp32-FMA
    kernel oflow_flow_head2_tiled_s32, FLOW_HEAD_MODE "tiled")
    against the reference's own flows for the same 8 pairs (tests/golden/raft_e2e_batch.npz), every pair."""
    from optical_flow import _native

    g = golden("raft_e2e_batch")
    b, h, w, iters, s, seed = (int(v) for v in g[f"{tag}_cfg"])
    img0, img1 = synthetic.synthetic_pair(b, h, w, seed=seed)
    chk = np.stack([[float(x.double().sum()), float((x.double() ** 2).sum()), float(x.abs().max())] for x in (img0, img1)])
    assert np.array_equal(chk, g[f"{tag}_img_checksum"])
    padder = InputPadder(img0.shape, mode=str(g[f"{tag}_mode"]))
    p0, p1 = (x.to(DEV) for x in padder.pad(img0, img1))
    model = _model(RAFT)
    assert model.pair_lanes == 2 and model.update_impl == "split" and model.encoder_impl == "split"
    lh, lw = p0.shape[-2] // 8, p0.shape[-1] // 8
    assert b * lh * lw > _native.FLOW_HEAD2_MAX_PIXELS  # the conv flow head, not the small-grid FMA kernel
    with torch.inference_mode():
        low, up = model(p0, p1, iters=iters, test_mode=True)
    up = padder.unpad(up)[..., ::s, ::s]
    for k in range(b):
        ml, xl = _epe(low[k : k + 1], g[f"{tag}_low"][k : k + 1])
        mu, xu = _epe(up[k : k + 1], g[f"{tag}_up"][k : k + 1])
        print(f"{tag} pair {k}: low EPE mean {ml:.2e} max {xl:.2e}; up EPE mean {mu:.2e} max {xu:.2e}")
        assert ml <= 1e-4 and mu <= 1e-4, (k, ml, mu)
        assert xl <= 1e-3 and xu <= 1e-3, (k, xl, xu)


def test_product_matches_oracle_on_gpu():
    """Same GPU convolutions, HIP correlation vs ATen correlation: isolates the kernels' contribution."""
    img0, img1 = synthetic.synthetic_pair(2, 436, 1024, seed=1)
    padder = InputPadder(img0.shape)
    p0, p1 = (x.to(DEV) for x in padder.pad(img0, img1))
    prod, orac = _model(RAFT), _model(oraft.RAFT)
    with torch.inference_mode():
        lo_p, up_p = prod(p0, p1, iters=12, test_mode=True)
        lo_o, up_o = orac(p0, p1, iters=12, test_mode=True)
    e = torch.norm(up_p - up_o, dim=1)
    print(f"product vs oracle-on-GPU: EPE mean {float(e.mean()):.2e} max {float(e.max()):.2e}")
    assert float(e.mean()) <= 1e-4 and float(e.max()) <= 1e-3


def test_train_mode_returns_all_predictions():
    img0, img1 = synthetic.synthetic_pair(1, 128, 128, seed=3)
    model = _model(RAFT)
    with torch.inference_mode():
        preds = model(img0.to(DEV), img1.to(DEV), iters=3)
        _, up = model(img0.to(DEV), img1.to(DEV), iters=3, test_mode=True)
    assert isinstance(preds, list) and len(preds) == 3
    assert torch.equal(preds[-1], up)


@pytest.mark.parametrize("lookup", ["joined", "lane"])
@pytest.mark.parametrize("b", [2, 3, 8])
def test_pair_lanes_equal_single_lane(lookup, b):
    """The split update loop on two pair lanes (streams) gives the single-lane results bit for bit (odd batches:
    ragged halves), in test mode and as the per-iteration prediction list."""
    img0, img1 = synthetic.synthetic_pair(2, 128, 160, seed=5)
    reps = -(-b // 2)
    p0 = img0.repeat(reps, 1, 1, 1)[:b].to(DEV)
    p1 = img1.repeat(reps, 1, 1, 1)[:b].to(DEV)
    p1[-1] = torch.roll(p1[-1], 3, dims=-1)  # distinct last pair
    model = _model(RAFT)
    outs = {}
    with torch.inference_mode():
        for lanes in (1, 2):
            model.pair_lanes, model.pair_lookup = lanes, lookup
            outs[lanes] = (model(p0, p1, iters=4, test_mode=True), model(p0, p1, iters=3))
    (lo1, up1), preds1 = outs[1]
    (lo2, up2), preds2 = outs[2]
    assert torch.equal(lo1, lo2) and torch.equal(up1, up2)
    assert len(preds1) == len(preds2) == 3 and all(torch.equal(a, c) for a, c in zip(preds1, preds2))


def test_pair_lanes_equal_single_lane_across_flow_head_threshold():
    """3 Sintel-size pairs (55x128 grid: 21120 px for the batch, 7040 / 14080 per lane) straddle the flow head's
    kernel choice (FLOW_HEAD2_MAX_PIXELS): the choice is made once per forward from the whole batch, so two lanes
    still give the single-lane flows bit for bit."""
    from optical_flow import _native

    b = 3
    assert b * 55 * 128 >= _native.FLOW_HEAD2_MAX_PIXELS > 2 * 55 * 128
    img0, img1 = synthetic.synthetic_pair(b, 440, 1024, seed=9)
    p0, p1 = img0.to(DEV), img1.to(DEV)
    model = _model(RAFT)
    outs = {}
    with torch.inference_mode():
        for lanes in (1, 2):
            model.pair_lanes = lanes
            outs[lanes] = model(p0, p1, iters=3, test_mode=True)
    assert torch.equal(outs[1][0], outs[2][0]) and torch.equal(outs[1][1], outs[2][1])


def test_fused_update_matches_module_update_block():
    """FusedUpdate (fused bias/activation/GRU kernels, merged z|r convolution, persistent [h | x] buffers) against
    the nn.Module update block on the same GPU, two steps so the carried state is checked too."""
    from model.update import FusedUpdate

    model = _model(RAFT)
    block = model.update_block
    b, h, w = 2, 24, 40
    g = lambda s, shape, std: torch.from_numpy(synthetic.hash_normal(s, shape, std)).to(DEV)
    net, inp = torch.tanh(g(1, (b, 128, h, w), 1.0)), torch.relu(g(2, (b, 128, h, w), 1.0))
    corr1, corr2 = g(3, (b, 324, h, w), 2.0), g(4, (b, 324, h, w), 2.0)
    flow1, flow2 = g(5, (b, 2, h, w), 3.0), g(6, (b, 2, h, w), 3.0)
    with torch.inference_mode():
        n1, m1, d1 = block(net, inp, corr1, flow1)
        n2, m2, d2 = block(n1, inp, corr2, flow2)
        runner = FusedUpdate(block, net, inp)
        f1 = runner.step(corr1, flow1)
        f2 = runner.step(corr2, flow2)
    for ref, got in zip((n1, m1, d1, n2, m2, d2), (*f1, *f2)):
        err = float((ref - got).abs().max())
        assert err <= 1e-4 * max(1.0, float(ref.abs().max())), err


class _FixedCorr:
    """Stands in for CorrBlock: hands the given lookup outputs to SplitUpdate (as NHWC rows) in order."""

    def __init__(self, corrs):
        self.corrs = list(corrs)

    def lookup_nhwc(self, coords, out):
        b, _, h, w = coords.shape
        out.view(b, h, w, -1).copy_(self.corrs.pop(0).permute(0, 2, 3, 1))
        return out


def test_split_update_matches_module_update_block():
    """SplitUpdate (split-fp16 convolutions, fused GRU / motion / flow-head epilogues, in-place coords) against the
    nn.Module update block (MIOpen fp32) on the same GPU, two steps so the carried state is checked too."""
    from model.update import SplitUpdate
    from model.utils import coords_grid

    model = _model(RAFT)
    block = model.update_block
    b, h, w = 2, 24, 40
    g = lambda s, shape, std: torch.from_numpy(synthetic.hash_normal(s, shape, std)).to(DEV)
    cnet_out = g(1, (b, 256, h, w), 1.0)
    net, inp = torch.tanh(cnet_out[:, :128]), torch.relu(cnet_out[:, 128:])
    corr1, corr2 = g(3, (b, 324, h, w), 2.0), g(4, (b, 324, h, w), 2.0)
    coords0 = coords_grid(b, h, w, device=DEV)
    coords1 = coords0 + g(5, (b, 2, h, w), 3.0)
    with torch.inference_mode():
        n1, m1, d1 = block(net, inp, corr1, coords1 - coords0)
        c1 = coords1 + d1
        n2, m2, d2 = block(n1, inp, corr2, c1 - coords0)
        c2 = c1 + d2
        runner = SplitUpdate(block, cnet_out.contiguous(), 128)
        cc = coords1.clone()
        fake = _FixedCorr([corr1, corr2])
        s1 = runner.step(fake, cc, need_mask=True)
        cc1 = cc.clone()
        h1 = runner.hm.view(b, h, w, 128).permute(0, 3, 1, 2).clone()
        s2 = runner.step(fake, cc, need_mask=True)
        h2 = runner.hm.view(b, h, w, 128).permute(0, 3, 1, 2)
    for what, ref, got in (("net1", n1, h1), ("mask1", m1, s1), ("coords1", c1, cc1), ("net2", n2, h2), ("mask2", m2, s2), ("coords2", c2, cc)):
        err = float((ref - got).abs().max())
        print(f"{what}: max |d| {err:.2e}")
        assert err <= 1e-4 * max(1.0, float(ref.abs().max())), (what, err)


@pytest.mark.parametrize("norm", ["instance", "batch"])
@pytest.mark.parametrize("b,h,w", [(2, 128, 160), (2, 440, 1024)])
def test_split_encoder_matches_module(norm, b, h, w):
    """SplitEncoder (split-fp16 convs, fp64-merged instance-norm statistics / folded eval batch norm, space-to-depth
    stride-2 stages) against the nn.Module encoder (MIOpen fp32) on the same GPU."""
    from model.extractor import BasicEncoder, SplitEncoder

    model = _model(RAFT)
    enc = model.fnet if norm == "instance" else model.cnet
    if norm == "batch":  # non-trivial running statistics and affine parameters
        g = torch.Generator().manual_seed(1)
        for m in enc.modules():
            if isinstance(m, torch.nn.BatchNorm2d):
                m.running_mean.copy_(torch.randn(m.num_features, generator=g) * 0.1)
                m.running_var.copy_(torch.rand(m.num_features, generator=g) + 0.5)
                m.weight.data.copy_(torch.rand(m.num_features, generator=g) + 0.5)
                m.bias.data.copy_(torch.randn(m.num_features, generator=g) * 0.1)
    img0, img1 = synthetic.synthetic_pair(b, h, w, seed=2)
    x = (2 * (img0.to(DEV) / 255.0) - 1.0).contiguous()
    with torch.inference_mode():
        ref = enc(x)
        got = SplitEncoder(enc)(x)
    err = float((got - ref).abs().max())
    scale = float(ref.abs().max())
    print(f"{norm} {b}x{h}x{w}: max |d| {err:.2e} (max |ref| {scale:.2f})")
    assert got.shape == ref.shape
    assert err <= 1e-4 * max(1.0, scale), err


@pytest.mark.parametrize("norm", ["instance", "batch"])
@pytest.mark.parametrize("b,h,w", [(2, 128, 160), (1, 440, 1024), (3, 72, 88)])
def test_split_encoder_stem_from_image_bit_identical(norm, b, h, w):
    """The stem conv building its 7x7/2 patch operand from the staged image window (OFLOW_IN_IMG7S2) gives the patch
    matrix path's encoder output bit for bit (same operand values, same k order): ragged 4x32 tiles (72x88 input ->
    36x44 stem output), image borders (zero padding), both norms."""
    from model.extractor import SplitEncoder

    model = _model(RAFT)
    enc = model.fnet if norm == "instance" else model.cnet
    img0, _ = synthetic.synthetic_pair(b, h, w, seed=4)
    x = (2 * (img0.to(DEV) / 255.0) - 1.0).contiguous()
    with torch.inference_mode():
        a = SplitEncoder(enc)(x)
        c = SplitEncoder(enc)(x, stem_from_image=True)
        sa = SplitEncoder(enc)(x, split_out=True)
        sc = SplitEncoder(enc)(x, split_out=True, stem_from_image=True)
    assert torch.equal(a, c) and torch.equal(sa, sc)


@pytest.mark.parametrize("shape", [(2, 55, 128), (1, 1, 1), (3, 7, 33), (1, 47, 156)])
def test_convex_upsample_matches_oracle(shape):
    """RAFT.upsample_flow on the GPU (one fused kernel, csrc/upsample.hip) vs the reference formula (raft.py:73-85) on
    the CPU: softmax over the 9 neighbours, unfold with zero padding at every border, permute/reshape order."""
    b, h, w = shape
    flow = torch.from_numpy(synthetic.hash_normal(21, (b, 2, h, w), 6.0))
    mask = torch.from_numpy(synthetic.hash_normal(22, (b, 576, h, w), 3.0))
    ref = oraft.upsample_flow(flow, mask)
    with torch.inference_mode():
        got = RAFT.upsample_flow(flow.to(DEV), mask.to(DEV)).cpu()
    assert got.shape == ref.shape == (b, 2, 8 * h, 8 * w)
    tol = 1e-5 * float(8 * flow.abs().max()) + 1e-6
    assert float((got - ref).abs().max()) <= tol


@pytest.mark.parametrize("sigma", [0.0, 3.0, 20.0])
def test_corr_backward_matches_oracle(sigma):
    """CorrBlock under autograd (native lookup transpose + pyramid-gradient fold + bmm) vs the reference's ATen
    composition (corr.py:38-87, utils.py:64-80) differentiated on the CPU: two lookups, fmap gradients."""
    from model import CorrBlock
    from oracle import corr as ocorr

    g = torch.Generator().manual_seed(int(sigma) + 11)
    b, c, h, w = 2, 32, 24, 33
    f1 = torch.randn(b, c, h, w, generator=g)
    f2 = torch.randn(b, c, h, w, generator=g)
    cs = [ocorr.coords_grid(b, h, w) + torch.randn(b, 2, h, w, generator=g) * sigma for _ in range(2)]
    rs = [torch.randn(b, 4 * 81, h, w, generator=g) for _ in range(2)]

    a1, a2 = f1.clone().requires_grad_(), f2.clone().requires_grad_()
    pyr = ocorr.corr_pyramid(a1, a2, 4)
    loss = sum((ocorr.corr_lookup(pyr, co, 4) * r).sum() for co, r in zip(cs, rs))
    loss.backward()

    d1, d2 = f1.to(DEV).requires_grad_(), f2.to(DEV).requires_grad_()
    cb = CorrBlock(d1, d2)
    lossd = sum((cb(co.to(DEV)) * r.to(DEV)).sum() for co, r in zip(cs, rs))
    lossd.backward()
    for ref, got in ((a1.grad, d1.grad), (a2.grad, d2.grad)):
        err = float((got.cpu() - ref).abs().max())
        assert err <= 1e-4 * float(ref.abs().max()) + 1e-5, err


def test_raft_training_gradients_match_oracle():
    """One training step's gradients (the reference's sequence loss, raft.py:149-175 / loss gamma 0.8) through the
    product RAFT on the GPU -- CorrBlock on the native backward kernels, convs on ATen -- vs the oracle composition
    (pure ATen) on the same GPU."""
    img0, img1 = synthetic.synthetic_pair(1, 128, 128, seed=5)
    target = torch.from_numpy(synthetic.hash_normal(31, (1, 2, 128, 128), 2.0)).to(DEV)
    grads = []
    for cls in (RAFT, oraft.RAFT):
        model = _model(cls)
        model.train()
        for m in model.modules():  # eval-mode batch norm: pairs independent, like the fixtures
            if isinstance(m, torch.nn.BatchNorm2d):
                m.eval()
        preds = model(img0.to(DEV), img1.to(DEV), iters=3)
        loss = sum(0.8 ** (len(preds) - i - 1) * (p - target).abs().mean() for i, p in enumerate(preds))
        loss.backward()
        grads.append({k: p.grad.detach().clone() for k, p in model.named_parameters() if p.grad is not None})
    prod, orac = grads
    assert set(prod) == set(orac)
    for k in ("fnet.conv1.weight", "fnet.layer3.1.conv2.weight", "update_block.gru.convz1.weight", "cnet.conv2.weight"):
        rel = float((prod[k] - orac[k]).norm() / orac[k].norm())
        assert rel <= 1e-3, (k, rel)


def test_graphed_forward_equals_eager():
    """model/graph.py: the forward replayed from a HIP graph (batch 1, 24 iterations: predict.py's case) gives the
    eager forward's flows bit for bit, also after new inputs are copied in."""
    from model.graph import GraphedRAFT

    model = _model(RAFT)
    pairs = [synthetic.synthetic_pair(1, 128, 160, seed=s) for s in (21, 22)]
    padder = InputPadder(pairs[0][0].shape)
    p = [[x.to(DEV) for x in padder.pad(a, b)] for a, b in pairs]
    with torch.inference_mode():
        g = GraphedRAFT(model, p[0][0], p[0][1], iters=24)
        for a, b in p:
            lo_e, up_e = model(a, b, iters=24, test_mode=True)
            lo_g, up_g = g(a, b)
            assert torch.equal(lo_g, lo_e) and torch.equal(up_g, up_e)


def test_graphed_multi_pair_forward_equals_eager_two_lanes():
    """GraphedRAFT on a multi-pair batch (3 pairs, above the flow-head threshold: the conv flow head) is captured with
    two pair lanes (without the lanes' side streams, whose nested fork crashes hipStreamEndCapture) and replays the
    eager two-lane forward's flows bit for bit; the model's settings are restored after the capture."""
    from model.graph import GraphedRAFT

    model = _model(RAFT)
    assert model.pair_lanes == 2
    a0, a1 = synthetic.synthetic_pair(3, 436, 1024, seed=31)  # 3 x 55 x 128 = 21120 px: conv flow head, two lanes
    padder = InputPadder(a0.shape)
    p0, p1 = (x.to(DEV) for x in padder.pad(a0, a1))
    with torch.inference_mode():
        g = GraphedRAFT(model, p0, p1, iters=6)
        assert model.pair_lanes == 2 and getattr(model.update_block, "split_streams", True)
        lo_e, up_e = model(p0, p1, iters=6, test_mode=True)
        lo_g, up_g = g(p0, p1)
        assert torch.equal(lo_g, lo_e) and torch.equal(up_g, up_e)


def test_graphed_forward_timing_event_nodes():
    """bench.py's graph mode: a recorder with native timing events ({'_native': True}) given to GraphedRAFT is active
    during the capture only; its event pairs around the fused lookup + convc1 and pyramid launches become event-record
    nodes of the graph, re-recorded by every replay: after a replay each pair reads a positive duration (the launch's),
    one pair per lane and iteration, and the flows still equal the eager forward's."""
    from model.graph import GraphedRAFT
    from optical_flow import _native

    model = _model(RAFT)
    a0, a1 = synthetic.synthetic_pair(3, 436, 1024, seed=33)
    padder = InputPadder(a0.shape)
    p0, p1 = (x.to(DEV) for x in padder.pad(a0, a1))
    rec = {"_native": True}
    with torch.inference_mode():
        g = GraphedRAFT(model, p0, p1, iters=4, recorder=rec)
        assert _native._recorder is None  # restored after the capture
        lo_g, up_g = g(p0, p1)
        torch.cuda.synchronize()
        lk = rec["corr_lookup_convc1"]
        assert len(lk) == 4 * 2  # iterations x pair lanes
        first = [a.elapsed_time(b) for a, b in lk]
        assert all(0.0 < t < 50.0 for t in first), first
        assert len(rec["corr_pyramid"]) == 1 and rec["corr_pyramid"][0][0].elapsed_time(rec["corr_pyramid"][0][1]) > 0
        g(p0, p1)  # a second replay re-records the same events
        torch.cuda.synchronize()
        assert all(0.0 < a.elapsed_time(b) < 50.0 for a, b in lk)
        lo_e, up_e = model(p0, p1, iters=4, test_mode=True)
    assert torch.equal(lo_g, lo_e) and torch.equal(up_g, up_e)


@pytest.mark.parametrize("where", ["images", "convc1", "convc2"])
def test_range_guard_raises_on_split_overflow(where):
    """The split-fp16 range guard (oflow_set_range_flag): an activation whose fp16 hi half overflows (|x| >= 65520) sets
    the device flag inside the kernel that splits it, and the forward raises RuntimeError -- with no per-convolution
    check. Injected three ways: huge input frames (cnet's stem output, batch norm folded), convc1 weights x 1e6 (the
    fused lookup + convc1 epilogue), convc2 weights x 1e6 (a conv_s32 epilogue's S32 store). A normal forward
    afterwards runs (the flag was cleared) and matches its earlier output bit for bit."""
    img0, img1 = synthetic.synthetic_pair(2, 128, 160, seed=6)
    p0, p1 = img0.to(DEV), img1.to(DEV)
    model = _model(RAFT)
    with torch.inference_mode():
        ref = model(p0, p1, iters=4, test_mode=True)
    bad = _model(RAFT)
    bad.range_guard = "sync"
    a0, a1 = p0, p1
    if where == "images":
        a0, a1 = p0 * 1e6, p1 * 1e6
    else:
        w = getattr(bad.update_block.encoder, where).weight
        with torch.no_grad():
            w.mul_(1e6)
        bad.invalidate_weight_caches()
    with torch.inference_mode():
        with pytest.raises(RuntimeError, match="fp16 range"):
            bad(a0, a1, iters=4, test_mode=True)
        got = model(p0, p1, iters=4, test_mode=True)  # flag cleared: a valid forward does not raise
    assert torch.equal(got[0], ref[0]) and torch.equal(got[1], ref[1])


def test_range_guard_deferred_mode():
    """range_guard = "deferred" (the default): the forward does not wait for the flag; check_range() raises, and so
    does a later forward once the GPU has finished the overflowing one; GraphedRAFT replays are guarded the same way."""
    from model.graph import GraphedRAFT

    img0, img1 = synthetic.synthetic_pair(1, 128, 160, seed=6)
    p0, p1 = img0.to(DEV), img1.to(DEV)
    bad = _model(RAFT)
    assert bad.range_guard == "deferred"
    with torch.inference_mode():
        bad(p0 * 1e6, p1 * 1e6, iters=2, test_mode=True)
        with pytest.raises(RuntimeError, match="fp16 range"):
            bad.check_range()
        bad.check_range()  # cleared
        bad(p0 * 1e6, p1 * 1e6, iters=2, test_mode=True)
        torch.cuda.synchronize()
        with pytest.raises(RuntimeError, match="fp16 range"):
            bad(p0, p1, iters=2, test_mode=True)  # reports the earlier forward
        bad.check_range(DEV)
        g = GraphedRAFT(bad, p0, p1, iters=2)
        g(p0, p1)
        bad.check_range(DEV)
        g(p0 * 1e6, p1 * 1e6)
        with pytest.raises(RuntimeError, match="fp16 range"):
            bad.check_range(DEV)


def test_range_snapshot_per_forward():
    """Each GPU inference forward's own range status (RAFT.last_range_snapshot, oflow_range_flag_exchange: the flag read
    and cleared in one device-side exchange after the forward's kernels): an overflowing forward's snapshot reports
    True; the next forward (deferred mode) first raises for it, and a valid forward after that reports False with
    nothing left set on the device."""
    img0, img1 = synthetic.synthetic_pair(1, 128, 160, seed=6)
    p0, p1 = img0.to(DEV), img1.to(DEV)
    m = _model(RAFT)
    with torch.inference_mode():
        m(p0 * 1e6, p1 * 1e6, iters=2, test_mode=True)
        bad = m.last_range_snapshot
        assert bad.overflowed()
        with pytest.raises(RuntimeError, match="fp16 range"):
            m(p0, p1, iters=2, test_mode=True)  # reports the earlier forward before running
        m(p0, p1, iters=2, test_mode=True)
        good = m.last_range_snapshot
        assert good is not bad and not good.overflowed()
        m.check_range(DEV)  # nothing left set


def test_forwards_in_flight_on_two_streams_equal_sequential():
    """Pipelined steps (bench.py --inflight): forwards issued back to back from two streams -- each with its own side
    and lane streams, the packed-weight caches shared behind an event -- give the flows of sequential forwards bit for
    bit, including the very first forward on the second stream (weights packed by the first)."""
    img0, img1 = synthetic.synthetic_pair(3, 128, 160, seed=8)
    p0, p1 = img0.to(DEV), img1.to(DEV)
    q0, q1 = torch.roll(p0, 5, dims=-1), torch.roll(p1, 5, dims=-1)
    model = _model(RAFT)
    with torch.inference_mode():
        ref_a = model(p0, p1, iters=6, test_mode=True)
        ref_b = model(q0, q1, iters=6, test_mode=True)
        torch.cuda.synchronize()
        fresh = _model(RAFT)  # empty caches: the second stream's first forward finds weights packed on the first
        s = [torch.cuda.current_stream(), torch.cuda.Stream()]
        outs = []
        for i in range(4):
            with torch.cuda.stream(s[i % 2]):
                outs.append(fresh(*((p0, p1) if i % 2 == 0 else (q0, q1)), iters=6, test_mode=True))
        torch.cuda.synchronize()
    for i, (lo, up) in enumerate(outs):
        ref = ref_a if i % 2 == 0 else ref_b
        assert torch.equal(lo, ref[0]) and torch.equal(up, ref[1]), i


@pytest.mark.parametrize("shape", [(3, 3, 68, 128), (3, 3, 67, 129)])  # vector and scalar kernel
def test_normalize_images_bit_identical_to_reference(shape):
    """oflow_normalize_images_f32 (RAFT.forward's input scaling, raft.py:104-105, both frames in one kernel) against the
    reference's `2 * (x / 255.0) - 1.0` computed on the CPU (as the reference runs): bit-identical over [0, 255] values
    and extremes. (ATen on the GPU divides by fl(1/255)-multiplication and differs by 1 ulp: profiles/r04/s36_div.log.)"""
    from optical_flow import _native as N

    g = torch.Generator().manual_seed(3)
    x0 = torch.rand(*shape, generator=g) * 255
    x1 = torch.randint(0, 256, shape, generator=g).float()
    x1.view(-1)[:6] = torch.tensor([0.0, 255.0, 1e-30, -0.0, 127.5, 3e38])
    y0, y1 = N.normalize_images(x0.to(DEV), x1.to(DEV))
    assert torch.equal(y0.cpu(), 2 * (x0 / 255.0) - 1.0) and torch.equal(y1.cpu(), 2 * (x1 / 255.0) - 1.0)


@pytest.mark.parametrize("shape,mode", [((8, 3, 436, 1024), "sintel"), ((2, 3, 375, 1242), "kitti"),
                                        ((1, 3, 61, 97), "sintel"), ((3, 2, 48, 64), "kitti")])
def test_input_padder_native_pad_equals_f_pad(shape, mode):
    """InputPadder.pad on GPU frames (oflow_replicate_pad_f32, all frames in one launch) against F.pad(mode='replicate')
    (utils.py:38-61): bit-exact, both modes, ragged sizes, already-aligned sizes."""
    import torch.nn.functional as F

    g = torch.Generator().manual_seed(shape[2])
    x0, x1 = (torch.rand(*shape, generator=g).to(DEV) * 255 for _ in range(2))
    padder = InputPadder(shape, mode=mode)
    p0, p1 = padder.pad(x0, x1)
    assert torch.equal(p0, F.pad(x0, padder._pad, mode="replicate"))
    assert torch.equal(p1, F.pad(x1, padder._pad, mode="replicate"))
    assert torch.equal(padder.unpad(p0), x0)
