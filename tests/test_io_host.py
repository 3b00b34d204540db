"""Inference I/O on the host, no GPU: the oracle's flow2rgb and file payloads against the
goldens the reference produced (tests/golden/io_small.npz, gen_goldens.py io), the file writers/readers on host
arrays byte-for-byte, and the reference's error behaviour (tests/io/test_read_write.py,
tests/visualization/test_flow2rgb.py). The product's flow2rgb has no CPU path: a CPU tensor raises."""
import numpy as np
import pytest
import torch

import optical_flow
from optical_flow.io import read, write
from optical_flow.io.middlebury import read_middleburry
from oracle import io as oio

# (clip, max_norm, invert_y) of each golden tag (gen_goldens.py IO_OPTIONS)
OPTIONS = {
    "d": (None, None, False),
    "c1": (1.0, None, False),
    "c50": (50.0, None, False),
    "cpos": ((0.0, 50.0), None, False),
    "m30": (None, 30.0, False),
    "inv": (None, None, True),
    "all": (20.0, 8.0, True),
}


@pytest.fixture(scope="module")
def io_golden(golden):
    return golden("io_small")


def test_oracle_flow2rgb_matches_reference_goldens(io_golden):
    keys = [k for k in io_golden if k.startswith("rgb_")]
    assert len(keys) == 3 * (2 * len(OPTIONS) + 3)
    for k in keys:
        _, name, method, tag = k.split("_")
        clip, max_norm, inv = OPTIONS[tag]
        got = oio.flow2rgb(io_golden[f"flow_{name}"], method, clip, max_norm, inv)
        # one fp32 op per reference op: equal up to a 1-ulp libm difference
        np.testing.assert_allclose(got, io_golden[k], rtol=0, atol=1e-6, err_msg=k)


def test_oracle_payloads_match_reference_file_bytes(io_golden):
    f = io_golden["flow_s"][1]
    assert oio.flo_bytes(f) == io_golden["bytes_flo"].tobytes()
    assert oio.pfm_bytes(f) == io_golden["bytes_pfm"].tobytes()


@pytest.mark.parametrize("fmt,key", [("middlebury", "bytes_flo"), ("pfm", "bytes_pfm")])
@pytest.mark.parametrize("kind", ["tensor", "numpy"])
def test_host_writer_bytes_equal_reference(tmp_path, io_golden, fmt, key, kind):
    f = io_golden["flow_s"][1]
    flow = torch.from_numpy(f.copy()) if kind == "tensor" else f.copy()
    path = tmp_path / "x"
    write(path, flow, fmt=fmt)
    assert path.read_bytes() == io_golden[key].tobytes()
    back = read(path, fmt=fmt)
    assert back.dtype == torch.float32 and back.device.type == "cpu"
    assert torch.equal(back, torch.from_numpy(f))


@pytest.mark.parametrize("fmt", ["middlebury", "pfm"])
def test_read_write_roundtrip_reference_case(tmp_path, fmt):
    # tests/io/test_read_write.py:24-37 on the CPU device
    flow = torch.rand(2, 5, 6) * 100
    write(tmp_path / "test", flow, fmt=fmt)
    loaded = read(tmp_path / "test", fmt=fmt)
    assert loaded.dtype == torch.float32 and loaded.shape == flow.shape and loaded.device == torch.device("cpu")
    assert torch.allclose(flow, loaded, atol=1e-8)


def test_kitti_needs_opencv_like_the_reference(tmp_path):
    pytest.importorskip("numpy")
    try:
        import cv2  # noqa: F401
    except ModuleNotFoundError:
        with pytest.raises(ModuleNotFoundError, match="opencv-python"):
            write(tmp_path / "k.png", torch.zeros(2, 3, 4), fmt="kitti")
        with pytest.raises(ModuleNotFoundError, match="opencv-python"):
            read(tmp_path / "k.png", fmt="kitti")
    else:  # pragma: no cover - cv2 is not in this image
        write(tmp_path / "k.png", torch.rand(2, 5, 6) * 100, fmt="kitti")


def test_errors_match_reference(tmp_path):
    with pytest.raises(ValueError, match="Unknown format"):
        write(tmp_path / "x", torch.zeros(2, 3, 4), fmt="png")
    with pytest.raises(ValueError, match="Unknown format"):
        read(tmp_path / "x", fmt="png")
    with pytest.raises(AssertionError):
        write(tmp_path / "x", torch.zeros(3, 3, 4))
    (tmp_path / "bad.flo").write_bytes(np.float32(1.0).tobytes() + b"\0" * 16)
    with pytest.raises(RuntimeError, match="Magic number"):
        read_middleburry(tmp_path / "bad.flo")
    (tmp_path / "bad.pfm").write_bytes(b"Pf\n2 2\n-1.0\n")
    with pytest.raises(RuntimeError, match="single-channel"):
        read(tmp_path / "bad.pfm", fmt="pfm")
    with pytest.raises(ValueError, match="Unknown method"):
        optical_flow.flow2rgb(torch.rand(4, 2, 5, 6), method="unknown")


def test_flow2rgb_has_no_cpu_fallback():
    with pytest.raises(RuntimeError, match="no CPU fallback"):
        optical_flow.flow2rgb(torch.rand(2, 5, 6))


def test_image_grid_layout_matches_save_image():
    # torchvision make_grid(nrow=8, padding=2, pad_value=0) + save_image's uint8 conversion, by hand
    import predict

    ims = [torch.full((3, 4, 5), v) for v in (0.1, 0.5, 1.0)]
    g = predict.image_grid(ims).numpy()
    assert g.shape == (4 + 4, 3 * 5 + 8, 3)
    for i, v in enumerate((0.1, 0.5, 1.0)):
        x0 = 2 + i * 7
        assert (g[2:6, x0:x0 + 5] == int(v * 255 + 0.5)).all()
    assert g[:2].max() == 0 and g[:, :2].max() == 0 and g[:, 7:9].max() == 0
