"""Inference I/O on the GPU through the C ABI: the flow2rgb kernels against the reference's
outputs (tests/golden/io_small.npz) and the oracle, the reference's own flow2rgb unit tests
(tests/visualization/test_flow2rgb.py) on the ROCm device, and the device-side file payloads byte-for-byte.

Tolerance: the colour maps are the reference's fp32 arithmetic op for op, but the GPU's atan2f/sqrtf may differ
from the host libm by an ulp; where that crosses a 1/255 quantisation step (baker's floor(255 c)) one channel
moves by 1/255. So: every element within 1/255 + 1e-6, and at most 0.1 % of elements (or 2) off by more than
1e-6."""
import numpy as np
import pytest
import torch

import optical_flow
from model import synthetic
from optical_flow import _native
from optical_flow.io import read, write
from oracle import io as oio

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)
OPTIONS = {
    "d": (None, None, False),
    "c1": (1.0, None, False),
    "c50": (50.0, None, False),
    "cpos": ((0.0, 50.0), None, False),
    "m30": (None, 30.0, False),
    "inv": (None, None, True),
    "all": (20.0, 8.0, True),
}


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    assert torch.cuda.is_available(), "GPU tests need a ROCm GPU"
    _native.load()


@pytest.fixture(scope="module")
def io_golden(golden):
    return golden("io_small")


def _close_rgb(got, ref, what):
    got = got.detach().cpu().numpy() if isinstance(got, torch.Tensor) else got
    ref = np.asarray(ref)
    assert got.shape == ref.shape, (what, got.shape, ref.shape)
    d = np.abs(got - ref)
    assert d.max() <= 1 / 255 + 1e-6, f"{what}: max |d| {d.max()}"
    assert (d > 1e-6).sum() <= max(2, 1e-3 * d.size), f"{what}: {(d > 1e-6).sum()} of {d.size} elements differ"


def test_flow2rgb_matches_reference_goldens(io_golden):
    for k in io_golden:
        if not k.startswith("rgb_"):
            continue
        _, name, method, tag = k.split("_")
        clip, max_norm, inv = OPTIONS[tag]
        flow = torch.from_numpy(io_golden[f"flow_{name}"]).to(DEV)
        _close_rgb(optical_flow.flow2rgb(flow, method, clip, max_norm, inv), io_golden[k], k)


@pytest.mark.parametrize("method", ["baker", "hsv", "meister"])
def test_colorwheel_matches_reference(io_golden, method, tmp_path):
    wheel = optical_flow.colorwheel(method, size=48, file=tmp_path / "w.png")
    assert wheel.device.type == "cuda"
    _close_rgb(wheel, io_golden[f"wheel_{method}"], f"wheel_{method}")
    assert (tmp_path / "w.png").stat().st_size > 0


@pytest.mark.parametrize("method", ["baker", "hsv", "meister"])
@pytest.mark.parametrize("shape", [(2, 2, 436, 1024), (1, 2, 1, 300), (3, 2, 17, 1)])
def test_flow2rgb_vs_oracle_large_and_ragged(method, shape):
    # a smooth field plus noise: every hue sector and both sides of rad == 1 (max_norm below the largest norm)
    b, _, h, w = shape
    yy, xx = np.meshgrid(np.linspace(-1, 1, h), np.linspace(-1, 1, w), indexing="ij")
    base = np.stack([xx * 30 - yy * 7, yy * 20 + xx * 5]).astype(np.float32)
    flow = base[None] + synthetic.hash_normal(960, shape, 2.0)
    for clip, max_norm in ((None, None), (25.0, 18.0)):
        got = optical_flow.flow2rgb(torch.from_numpy(flow).to(DEV), method, clip, max_norm)
        _close_rgb(got, oio.flow2rgb(flow, method, clip, max_norm), f"{method} {shape} clip={clip}")


@pytest.mark.parametrize("method", optical_flow.visualization.METHODS)
@pytest.mark.parametrize("shape", [[1, 2, 3, 4], [4, 2, 3, 4], [2, 3, 4]])
def test_flow2rgb_input_output_shape(method, shape):
    # tests/visualization/test_flow2rgb.py:47-55 on the GPU
    out = optical_flow.flow2rgb(torch.randn(*shape, device=DEV) * 100, method=method)
    expected = list(shape)
    expected[-3] = 3
    assert list(out.shape) == expected and out.dtype == torch.float32 and out.device.type == "cuda"


@pytest.mark.parametrize("method", optical_flow.visualization.METHODS)
def test_flow2rgb_numpy_conversion(method):
    # tests/visualization/test_flow2rgb.py:58-64: a NumPy array goes to the current ROCm device
    out = optical_flow.flow2rgb(np.random.uniform(-100, 100, size=(4, 2, 5, 5)), method=method)
    assert isinstance(out, torch.Tensor) and list(out.shape) == [4, 3, 5, 5] and out.device.type == "cuda"


@pytest.mark.parametrize("method", optical_flow.visualization.METHODS)
@pytest.mark.parametrize("clip", [1.0, 50.0])
def test_flow2rgb_clip(method, clip):
    # tests/visualization/test_flow2rgb.py:67-76
    flow = torch.randn(4, 2, 5, 6, device=DEV) * 100
    out0 = optical_flow.flow2rgb(flow, method=method, clip=clip)
    out1 = optical_flow.flow2rgb(torch.clip(flow, -clip, clip), method=method, clip=None)
    assert torch.equal(out0, out1)
    assert 0 <= out0.min() <= out0.max() <= 1


@pytest.mark.parametrize("method", optical_flow.visualization.METHODS)
def test_flow2rgb_invert_y(method):
    # tests/visualization/test_flow2rgb.py:79-87 (the reference test compares baker outputs whatever `method` is)
    flow = torch.randn(4, 2, 5, 6, device=DEV)
    inverted = flow.clone()
    inverted[:, 1] *= -1
    assert torch.equal(optical_flow.flow2rgb(flow, method=method),
                       optical_flow.flow2rgb(inverted, method=method, invert_y=True))


@pytest.mark.parametrize("method", optical_flow.visualization.METHODS)
def test_flow2rgb_max_norm_scales(method):
    # max_norm = the largest norm reproduces the default; scaling flow and max_norm together is invariant
    flow = torch.randn(2, 2, 9, 11, device=DEV) * 10
    m = float(torch.norm(flow[0], dim=0).max())
    _close_rgb(optical_flow.flow2rgb(flow[:1], method=method),
               optical_flow.flow2rgb(flow[:1], method=method, max_norm=torch.tensor(m)).cpu().numpy(), method)
    a = optical_flow.flow2rgb(flow * 4, method=method, max_norm=40.0)
    b = optical_flow.flow2rgb(flow, method=method, max_norm=10.0)
    _close_rgb(a, b.cpu().numpy(), f"{method} scale")


@pytest.mark.parametrize("fmt,key", [("middlebury", "bytes_flo"), ("pfm", "bytes_pfm")])
def test_device_writer_bytes_equal_reference(tmp_path, io_golden, fmt, key):
    f = torch.from_numpy(io_golden["flow_s"][1]).to(DEV)
    write(tmp_path / "x", f, fmt=fmt)
    assert (tmp_path / "x").read_bytes() == io_golden[key].tobytes()
    back = read(tmp_path / "x", fmt=fmt)
    assert back.device.type == "cpu" and torch.equal(back, f.cpu())


@pytest.mark.parametrize("channels,flip", [(2, False), (3, True), (3, False)])
def test_flow_pack_layouts(channels, flip):
    flow = torch.randn(3, 2, 7, 300, device=DEV)
    got = _native.flow_pack(flow, channels, flip).cpu()
    ref = flow.cpu().permute(0, 2, 3, 1)
    if channels == 3:
        ref = torch.cat([ref, torch.zeros_like(ref[..., :1])], -1)
    if flip:
        ref = ref.flip(1)
    assert torch.equal(got, ref)


@pytest.mark.parametrize("fmt", ["middlebury", "pfm"])
def test_read_write_roundtrip_reference_case_gpu(tmp_path, fmt):
    # tests/io/test_read_write.py:9-37 on the cuda device
    flow = torch.rand(2, 5, 6, device=DEV) * 100
    write(tmp_path / "test", flow, fmt=fmt)
    loaded = read(tmp_path / "test", fmt=fmt)
    assert loaded.dtype == torch.float32 and loaded.shape == flow.shape and loaded.device == torch.device("cpu")
    assert torch.allclose(flow.cpu(), loaded, atol=1e-8)


def test_predict_pipeline_writes_reference_files(tmp_path):
    # methods/raft/predict.py:39-95: consecutive pairs -> {i:06d}.flo + {i:06d}.png grids
    import predict
    from PIL import Image
    from model import RAFT, InputPadder

    src = tmp_path / "frames"
    src.mkdir()
    frames = []
    for k in range(3):
        img, _ = synthetic.synthetic_pair(1, 131, 203, seed=20 + k)
        arr = img[0].permute(1, 2, 0).clamp(0, 255).to(torch.uint8).numpy()
        Image.fromarray(arr, "RGB").save(src / f"f{k}.png")
        frames.append(torch.from_numpy(arr).permute(2, 0, 1).float())
    n = predict.main(str(src), str(tmp_path / "out"), iters=3, eval_mode=True, num_workers=0)
    assert n == 2

    model = RAFT()
    model.load_state_dict(synthetic.synthetic_state_dict(model.state_dict()))
    model = model.to(DEV).eval()
    for i in range(2):
        img0, img1 = frames[i][None].to(DEV), frames[i + 1][None].to(DEV)
        padder = InputPadder(img0.shape)
        with torch.inference_mode():
            _, up = model(*padder.pad(img0, img1), iters=3, test_mode=True)
        flow = padder.unpad(up)[0]
        got = read(tmp_path / "out" / f"{i:06d}.flo")
        assert got.shape == (2, 131, 203)
        torch.testing.assert_close(got, flow.cpu(), rtol=0, atol=1e-5)
        png = np.array(Image.open(tmp_path / "out" / f"{i:06d}.png"))
        assert png.shape == (131 + 4, 3 * 203 + 8, 3)
        want = predict.image_grid([img0[0] / 255.0, img1[0] / 255.0, optical_flow.flow2rgb(flow)]).cpu().numpy()
        assert np.abs(png.astype(int) - want.astype(int)).max() <= 1


def test_predict_writes_nothing_for_an_overflowing_pair(tmp_path):
    """predict.py's writer checks each pair's own split-fp16 range snapshot (RAFT.last_range_snapshot) before writing:
    with convc1 weights scaled so that every forward overflows, the run raises and leaves no .flo / .png behind."""
    import predict
    from PIL import Image
    from model import RAFT

    src = tmp_path / "frames"
    src.mkdir()
    for k in range(2):
        img, _ = synthetic.synthetic_pair(1, 128, 160, seed=30 + k)
        Image.fromarray(img[0].permute(1, 2, 0).clamp(0, 255).to(torch.uint8).numpy(), "RGB").save(src / f"f{k}.png")
    model = RAFT()
    sd = synthetic.synthetic_state_dict(model.state_dict())
    sd["update_block.encoder.convc1.weight"] = sd["update_block.encoder.convc1.weight"] * 1e6
    torch.save(sd, tmp_path / "bad.pth")
    with pytest.raises(RuntimeError, match="fp16 range"):
        predict.main(str(src), str(tmp_path / "out"), checkpoint=str(tmp_path / "bad.pth"), iters=2, eval_mode=True,
                     num_workers=0)
    assert not list((tmp_path / "out").glob("*.flo")) and not list((tmp_path / "out").glob("*.png"))


def test_model_built_under_inference_mode(golden):
    # predict.py:39 builds the model inside @torch.inference_mode(): its weights are inference tensors (no
    # version counter), which the packed-weight caches must accept
    from model import RAFT, InputPadder

    g = golden("raft_e2e")
    b, h, w, iters, s, seed = (int(v) for v in g["small_cfg"])
    img0, img1 = synthetic.synthetic_pair(b, h, w, seed=seed)
    with torch.inference_mode():
        model = RAFT()
        model.load_state_dict(synthetic.synthetic_state_dict(model.state_dict()))
        model = model.to(DEV).eval()
        padder = InputPadder(img0.shape)
        _, up = model(*(x.to(DEV) for x in padder.pad(img0, img1)), iters=iters, test_mode=True)
    epe = torch.norm(padder.unpad(up).cpu() - torch.from_numpy(g["small_up"]), dim=1)
    assert float(epe.mean()) <= 1e-4 and float(epe.max()) <= 1e-3
