"""Pin the oracle against fixtures produced by the reference itself (tests/golden/gen_goldens.py) and against
the reference's own exact unit-test vectors (tests/operator/test_operator.py:6-132). CPU only."""
import numpy as np
import pytest
import torch

from model import synthetic
from oracle import corr as ocorr
from oracle import operator as oop
from oracle import raft as oraft


def _fmaps(g, tag):
    b, c, h, w = (int(v) for v in g[f"{tag}_shape"])
    f1, f2 = synthetic.synthetic_fmaps(b, c, h, w, stream=int(g[f"{tag}_stream"]))
    # the generator must still reproduce the exact inputs the fixture was made from
    for f, key in ((f1, "fmap1"), (f2, "fmap2")):
        a = f.double().numpy()
        np.testing.assert_array_equal(np.array([a.sum(), (a * a).sum(), np.abs(a).max()]), g[f"{tag}_{key}_checksum"])
    return f1, f2


@pytest.mark.parametrize("tag", ["a", "b"])
def test_corr_pyramid_matches_reference(golden, tag):
    g = golden("corr_small")
    f1, f2 = _fmaps(g, tag)
    pyr = ocorr.corr_pyramid(f1, f2, 4)
    for lvl, p in enumerate(pyr):
        ref = g[f"{tag}_pyr{lvl}"]
        assert p.shape == ref.shape
        np.testing.assert_allclose(p.numpy(), ref, rtol=1e-5, atol=1e-5)


def test_corr_lookup_matches_reference(golden):
    g = golden("corr_small")
    for tag in ("a", "b"):
        f1, f2 = _fmaps(g, tag)
        pyr = [torch.from_numpy(g[f"{tag}_pyr{lvl}"]) for lvl in range(4)]
        keys = [k for k in g if k.startswith(f"{tag}_coords_") and k != "a_coords_r2"]
        assert keys
        for k in keys:
            coords = torch.from_numpy(g[k])
            out = ocorr.corr_lookup(pyr, coords, 4)
            ref = g[k.replace("coords", "lookup")]
            np.testing.assert_allclose(out.numpy(), ref, rtol=0, atol=1e-5)
            # independent float64 pixel-space restatement, tolerance 1e-4 (§8(c))
            if tag == "a":
                o64 = ocorr.corr_lookup_f64([p.numpy() for p in pyr], coords.numpy(), 4)
                np.testing.assert_allclose(o64, ref, rtol=0, atol=1e-4)
    pyr3 = ocorr.corr_pyramid(*_fmaps(g, "a"), 3)
    out = ocorr.corr_lookup(pyr3, torch.from_numpy(g["a_coords_r2"]), 2)
    np.testing.assert_allclose(out.numpy(), g["a_lookup_r2_l3"], rtol=0, atol=1e-5)


def test_window_channel_order_q1():
    """Q1: channel l*81 + i*9 + j samples at (x + i - 4, y + j - 4)."""
    vol = torch.zeros(1, 1, 16, 16)
    vol[0, 0, 8 + 3, 8 + 1] = 1.0  # dy=+3, dx=+1 from centre (8, 8)
    coords = torch.tensor([8.0, 8.0]).view(1, 2, 1, 1)
    out = ocorr.corr_lookup([vol], coords, 4)
    assert int(out.view(-1).argmax()) == 5 * 9 + 7


def test_warp_matches_reference(golden):
    g = golden("warp_small")
    frame, flow = torch.from_numpy(g["frame"]), torch.from_numpy(g["flow"])
    for key in g:
        if key.startswith("warp_") and key != "warp_default":
            _, mode, pad, ac = key.split("_")
            out = oop.warp(frame, flow, mode, pad, bool(int(ac)))
            np.testing.assert_allclose(out.numpy(), g[key], rtol=0, atol=1e-4, err_msg=key)
    np.testing.assert_array_equal(oop.warp(frame, flow).numpy(), g["warp_default"])
    np.testing.assert_array_equal(oop.warp_grid(flow.permute(0, 2, 3, 1)).numpy(), g["grid"])
    fp = torch.from_numpy(g["flow_px"])
    np.testing.assert_allclose(oop.integrate(fp, 0.5 * fp, -0.25 * fp).numpy(), g["integrate_3"], atol=1e-4)


def test_reference_unit_vectors():
    """Exact vectors of the reference's own tests (tests/operator/test_operator.py:6-38, 63-132)."""
    img = torch.tensor([[[1.0, 2.0]]]).unsqueeze(0)
    flow = torch.tensor([[[1.0, 0.0]], [[0.0, 0.0]]]).unsqueeze(0)
    assert torch.equal(oop.warp(img, oop.normalize(flow)), torch.tensor([[[2.0, 2.0]]]).unsqueeze(0))
    img = torch.tensor([[[1.0], [2.0]]]).unsqueeze(0)
    flow = torch.tensor([[[0.0], [0.0]], [[1.0], [0.0]]]).unsqueeze(0)
    assert torch.equal(oop.warp(img, oop.normalize(flow)), torch.tensor([[[2.0], [2.0]]]).unsqueeze(0))
    flow = torch.tensor([[[1.0, 3.0], [2.0, 4.0]], [[-1.0, -2.0], [-3.0, -4.0]]]).unsqueeze(0)
    exp = 2 * torch.tensor(
        [
            [[1.0, 1.5, 2.5, 3.0], [1.25, 1.75, 2.75, 3.25], [1.75, 2.25, 3.25, 3.75], [2.0, 2.5, 3.5, 4.0]],
            [[-1.0, -1.25, -1.75, -2.0], [-1.5, -1.75, -2.25, -2.5], [-2.5, -2.75, -3.25, -3.5], [-3.0, -3.25, -3.75, -4.0]],
        ]
    ).unsqueeze(0)
    assert torch.equal(oop.resize(flow, scale_factor=2), exp)


def test_state_dict_layout_matches_reference_count():
    m = oraft.RAFT()
    sd = m.state_dict()
    assert len(sd) == 179
    assert sum(v.numel() for v in sd.values()) == 5_261_329


@pytest.mark.parametrize("tag", ["small", "kittimode"])
def test_raft_forward_matches_reference(golden, tag):
    g = golden("raft_e2e")
    b, h, w, iters, s, seed = (int(v) for v in g[f"{tag}_cfg"])
    torch.set_num_threads(max(1, torch.get_num_threads()))
    model = oraft.RAFT().eval()
    model.load_state_dict(synthetic.synthetic_state_dict(model.state_dict()))
    img0, img1 = synthetic.synthetic_pair(b, h, w, seed=seed)
    padder = oraft.InputPadder(img0.shape, mode=str(g[f"{tag}_mode"]))
    with torch.inference_mode():
        low, up = model(*padder.pad(img0, img1), iters=iters, test_mode=True)
    up = padder.unpad(up)[..., ::s, ::s]
    epe_low = oraft.end_point_error(low, torch.from_numpy(g[f"{tag}_low"]))
    epe_up = oraft.end_point_error(up, torch.from_numpy(g[f"{tag}_up"]))
    assert float(epe_low.mean()) <= 1e-4 and float(epe_low.max()) <= 1e-3
    assert float(epe_up.mean()) <= 1e-4 and float(epe_up.max()) <= 1e-3


@pytest.mark.parametrize("tag,pair", [("sintel8", 7), ("kitti8", 3)])
def test_batch_goldens_are_per_pair_reference_flows(golden, tag, pair):
    """raft_e2e_batch.npz (the benchmarked 8-pair batches, made by the reference itself): the frames are the
    repository's generator output (input checksums), and pair k of the batch equals the oracle's forward of that
    pair alone (synthetic_pair seeds pair k with seed + k) -- pairs are independent, so the batch golden pins every
    pair of the GPU's batched forward."""
    g = golden("raft_e2e_batch")
    b, h, w, iters, s, seed = (int(v) for v in g[f"{tag}_cfg"])
    assert b == 8 and iters == 12
    img0, img1 = synthetic.synthetic_pair(1, h, w, seed=seed + pair)
    model = oraft.RAFT().eval()
    model.load_state_dict(synthetic.synthetic_state_dict(model.state_dict()))
    padder = oraft.InputPadder(img0.shape, mode=str(g[f"{tag}_mode"]))
    with torch.inference_mode():
        low, up = model(*padder.pad(img0, img1), iters=iters, test_mode=True)
    up = padder.unpad(up)[..., ::s, ::s]
    epe_low = oraft.end_point_error(low, torch.from_numpy(g[f"{tag}_low"][pair : pair + 1]))
    epe_up = oraft.end_point_error(up, torch.from_numpy(g[f"{tag}_up"][pair : pair + 1]))
    assert float(epe_low.mean()) <= 1e-4 and float(epe_low.max()) <= 1e-3
    assert float(epe_up.mean()) <= 1e-4 and float(epe_up.max()) <= 1e-3


def test_batch_golden_input_checksums(golden):
    g = golden("raft_e2e_batch")
    for tag in ("sintel8", "kitti8"):
        b, h, w, iters, s, seed = (int(v) for v in g[f"{tag}_cfg"])
        img0, img1 = synthetic.synthetic_pair(b, h, w, seed=seed)
        chk = np.stack([[float(x.double().sum()), float((x.double() ** 2).sum()), float(x.abs().max())] for x in (img0, img1)])
        assert np.array_equal(chk, g[f"{tag}_img_checksum"]), tag


def test_hd_golden_inputs_and_oracle(golden):
    """raft_e2e_hd.npz (BASELINE configs[4]: one 1080x1920 pair, 12 iterations, made by the reference's dense fp32
    CPU path): the frames are the repository's generator output (input checksums), and the oracle's forward of the
    pair matches the reference's flows at the fp32 bar -- the oracle is pinned at the configs[4] size too."""
    g = golden("raft_e2e_hd")
    b, h, w, iters, s, seed = (int(v) for v in g["hd1_cfg"])
    assert (b, h, w, iters) == (1, 1080, 1920, 12)
    img0, img1 = synthetic.synthetic_pair(b, h, w, seed=seed)
    chk = np.stack([[float(x.double().sum()), float((x.double() ** 2).sum()), float(x.abs().max())] for x in (img0, img1)])
    assert np.array_equal(chk, g["hd1_img_checksum"])
    model = oraft.RAFT().eval()
    model.load_state_dict(synthetic.synthetic_state_dict(model.state_dict()))
    padder = oraft.InputPadder(img0.shape, mode=str(g["hd1_mode"]))
    with torch.inference_mode():
        low, up = model(*padder.pad(img0, img1), iters=iters, test_mode=True)
    up = padder.unpad(up)[..., ::s, ::s]
    epe_low = oraft.end_point_error(low, torch.from_numpy(g["hd1_low"]))
    epe_up = oraft.end_point_error(up, torch.from_numpy(g["hd1_up"]))
    assert float(epe_low.mean()) <= 1e-4 and float(epe_low.max()) <= 1e-3
    assert float(epe_up.mean()) <= 1e-4 and float(epe_up.max()) <= 1e-3
