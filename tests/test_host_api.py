"""Host-side logic of the drop-in API on CPU: no-fallback behaviour, the reference's operator unit tests,
padding, grids, and state_dict compatibility."""
import numpy as np
import pytest
import torch

import optical_flow
from model import RAFT, CorrBlock, InputPadder, bilinear_sampler, coords_grid, synthetic
from model.raft import strip_module
from oracle import corr as ocorr
from oracle import operator as oop
from oracle import raft as oraft


def test_hip_ops_refuse_cpu_tensors():
    f = torch.zeros(1, 8, 16, 16)
    with pytest.raises(RuntimeError, match="no CPU fallback"):
        CorrBlock(f, f)
    with pytest.raises(RuntimeError, match="no CPU fallback"):
        optical_flow.warp(torch.zeros(1, 3, 4, 4), torch.zeros(1, 2, 4, 4))
    with pytest.raises(RuntimeError, match="no CPU fallback"):
        bilinear_sampler(torch.zeros(2, 1, 4, 4), torch.zeros(2, 3, 3, 2))


def test_reference_operator_unit_tests():
    """tests/operator/test_operator.py:41-132 (scale/resize) — elementwise helpers run anywhere."""
    fx = torch.tensor([[[1.0, 3.0], [2.0, 4.0]]]).unsqueeze(0)
    fy = torch.tensor([[[-1.0, -2.0], [-3.0, -4.0]]]).unsqueeze(0)
    flow = torch.cat((fx, fy), 1)
    s = optical_flow.scale(flow, 2)
    assert torch.equal(s[:, 0:1], 2 * fx) and torch.equal(s[:, 1:2], 2 * fy)
    s = optical_flow.scale(flow, (3, -1))
    assert torch.equal(s[:, 0:1], 3 * fx) and torch.equal(s[:, 1:2], -1 * fy)
    flow = torch.tensor([[[1.0, 3.0], [2.0, 4.0]], [[-1.0, -2.0], [-3.0, -4.0]]]).unsqueeze(0)
    assert torch.equal(optical_flow.resize(flow, scale_factor=2), oop.resize(flow, scale_factor=2))
    exp = torch.tensor(
        [[[1.0, 3.0], [1.25, 3.25], [1.75, 3.75], [2.0, 4.0]], [[-1.0, -2.0], [-1.5, -2.5], [-2.5, -3.5], [-3.0, -4.0]]]
    ).unsqueeze(0)
    exp[:, 1] *= 2
    assert torch.equal(optical_flow.resize(flow, size=(4, 2)), exp)
    exp = torch.tensor(
        [[[1.0, 1.5, 2.5, 3.0], [2.0, 2.5, 3.5, 4.0]], [[-1.0, -1.25, -1.75, -2.0], [-3.0, -3.25, -3.75, -4.0]]]
    ).unsqueeze(0)
    exp[:, 0] *= 2
    assert torch.equal(optical_flow.resize(flow, size=(2, 4)), exp)
    f = torch.randn(2, 2, 7, 9)
    assert torch.equal(optical_flow.normalize(f), oop.normalize(f))
    assert torch.equal(optical_flow.denormalize(f), oop.denormalize(f))
    with pytest.raises(AssertionError):
        optical_flow.scale(torch.zeros(1, 3, 2, 2), 2.0)


def test_warp_grid_matches_oracle(golden):
    g = golden("warp_small")
    flow = torch.from_numpy(g["flow"]).permute(0, 2, 3, 1)
    np.testing.assert_array_equal(optical_flow.warp_grid(flow).numpy(), g["grid"])


@pytest.mark.parametrize("mode", ["sintel", "kitti", "chairs"])
@pytest.mark.parametrize("hw", [(436, 1024), (375, 1242), (128, 128), (150, 203)])
def test_input_padder_matches_oracle(mode, hw):
    x = torch.arange(2 * 3 * hw[0] * hw[1], dtype=torch.float32).view(2, 3, *hw)
    a, b = InputPadder(x.shape, mode=mode), oraft.InputPadder(x.shape, mode=mode)
    assert a._pad == b._pad
    (pa,) = a.pad(x)
    assert pa.shape[-2] % 8 == 0 and pa.shape[-1] % 8 == 0
    assert torch.equal(pa, b.pad(x)[0])
    assert torch.equal(a.unpad(pa), x)


def test_coords_grid():
    assert torch.equal(coords_grid(2, 5, 7), ocorr.coords_grid(2, 5, 7))


def test_state_dict_keys_match_oracle_and_reference_count():
    a, b = RAFT().state_dict(), oraft.RAFT().state_dict()
    assert list(a.keys()) == list(b.keys())
    assert all(a[k].shape == b[k].shape for k in a)
    assert len(a) == 179


def test_hparams_and_checkpoint_roundtrip(tmp_path):
    m = RAFT(corr_radius=4, iters=12)
    assert m.hparams.hidden_dim == 128 and m.hparams.corr_levels == 4
    sd = synthetic.synthetic_state_dict(m.state_dict())
    ck = tmp_path / "raft.ckpt"
    torch.save({"state_dict": sd, "hyper_parameters": dict(m.hparams)}, ck)
    m2 = RAFT.load_from_checkpoint(ck)
    assert all(torch.equal(m2.state_dict()[k], sd[k]) for k in sd)
    pth = tmp_path / "raft.pth"
    torch.save({"module." + k: v for k, v in sd.items()}, pth)
    m3 = RAFT.load_from_checkpoint(pth)
    assert all(torch.equal(m3.state_dict()[k], sd[k]) for k in sd)
    assert list(strip_module({"module.a": 1, "b": 2})) == ["a", "b"]


def test_synthetic_generators_are_deterministic():
    a0, a1 = synthetic.synthetic_pair(1, 40, 48, seed=2)
    b0, b1 = synthetic.synthetic_pair(1, 40, 48, seed=2)
    assert torch.equal(a0, b0) and torch.equal(a1, b1)
    assert float(a0.min()) >= 0 and float(a0.max()) <= 255 and torch.equal(a0, a0.round())
    # frame1(x) = frame0(x - (3, -1.5)): integer part of the shift checks exactly on the half-pixel lattice
    c0, c1 = synthetic.synthetic_pair(1, 40, 48, shift=(3.0, -2.0), seed=2)
    assert torch.equal(c1[..., 0:30, 10:40], c0[..., 2:32, 7:37])


def test_load_state_dict_drops_packed_weight_caches():
    """Parameters created under torch.inference_mode() have no version counter, so the split kernels' packed-weight
    caches (keyed by storage) must be dropped when new weights are loaded in place."""
    with torch.inference_mode():
        model = RAFT()
    mods = (model.fnet, model.cnet, model.update_block)
    for m in mods:
        m.__dict__["_split_weights"] = ("stale", {})
    with torch.inference_mode():
        model.load_state_dict(synthetic.synthetic_state_dict(model.state_dict()))
    assert all("_split_weights" not in m.__dict__ for m in mods)
    for m in mods:
        m.__dict__["_split_weights"] = ("stale", {})
    model.invalidate_weight_caches()
    assert all("_split_weights" not in m.__dict__ for m in mods)


def test_bench_batch_golden_and_step_epe(golden):
    """bench.py's parity leg (host logic): the benchmarked workloads find their reference-generated batch golden, and
    the EPE of the golden's own flows against itself is exactly 0 (per pair, strided full-res included)."""
    import bench

    for wl, tag in (("sintel", "sintel8"), ("kitti", "kitti8")):
        _, h, w, iters, _, _ = bench.WORKLOADS[wl]
        t, g = bench.batch_golden(wl, h, w, iters)
        assert t == tag and g is not None
        b, gh, gw, _, s, _ = (int(v) for v in g[f"{tag}_cfg"])
        low = torch.from_numpy(g[f"{tag}_low"])
        # a full-res flow whose stride-s samples are the golden's
        up = torch.zeros(b, 2, gh, gw)
        up[..., ::s, ::s] = torch.from_numpy(g[f"{tag}_up"])
        e = bench.step_epe((low, up), t, g, 8)
        assert e["pairs"] == 8 and e["low_max"] == 0.0 and e["up_max"] == 0.0
    assert bench.batch_golden("sintel", 436, 1024, 24) == (None, None)  # other iteration counts: no batch golden
    t, g = bench.batch_golden("hd", 1080, 1920, 12)  # configs[4]: the reference's 1080p pair
    assert t == "hd1" and tuple(int(v) for v in g["hd1_cfg"][:4]) == (1, 1080, 1920, 12)
    assert bench.batch_golden("hd", 1080, 1920, 24) == (None, None)


def test_cached_pack_keys_and_rebuilds():
    """The packed-weight cache (model.update.cached_pack): a hit returns the cached object, a new key rebuilds; on a
    CPU-only host no event is recorded."""
    from model.update import cached_pack

    m = torch.nn.Linear(2, 2)
    calls = []
    a = cached_pack(m, ("k", 1), lambda: calls.append(1) or {"w": 1})
    b = cached_pack(m, ("k", 1), lambda: calls.append(2) or {"w": 2})
    c = cached_pack(m, ("k", 2), lambda: calls.append(3) or {"w": 3})
    assert a is b and c == {"w": 3} and calls == [1, 3]


def test_conv_frag_pack_is_a_permutation():
    """ConvWeights.frag holds exactly the pack's halves, fragment-major: element (g, t, n, hl, k) of the pack at
    [g][t][n / 32][k / 16][hl][(k / 8) % 2][n % 32][k % 8]."""
    from optical_flow import _native as N

    g = torch.Generator().manual_seed(5)
    wt = torch.randn(96, 64, 3, 3, generator=g)
    cw = N.ConvWeights(wt, None, 128)
    f = cw.frag()
    assert f is cw.frag() and f.shape == (2, 9, 4, 2, 2, 2, 32, 8)
    p = cw.pack
    for (gg, t, n, hl, k) in [(0, 0, 0, 0, 0), (1, 8, 127, 1, 31), (0, 4, 33, 1, 9), (1, 2, 95, 0, 17)]:
        assert torch.equal(f[gg, t, n // 32, k // 16, hl, (k // 8) % 2, n % 32, k % 8], p[gg, t, n, hl, k])
