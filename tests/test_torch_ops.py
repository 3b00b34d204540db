"""``torch.ops.oflow`` (csrc/torch_ops.cpp): the operator library loads on the CPU, registers every op with a Meta
kernel (what torch.compile's fake tensors run), carries the autograd formulas of optical_flow/_ops.py, and refuses
CPU tensors. No kernel is launched here; the GPU half (values, torch.compile fullgraph) is in test_gpu_ops.py."""
import pytest
import torch

from optical_flow import _native, _ops

META = torch.device("meta")


def test_every_op_is_registered():
    _native.load()
    for name in _ops.OPS:
        op = getattr(torch.ops.oflow, name)
        assert op.default._schema.name == f"oflow::{name}"


def test_meta_shapes():
    _native.load()
    f = torch.empty(2, 64, 55, 128, device=META)
    pyr = torch.ops.oflow.corr_pyramid(f, f, 4)
    assert [tuple(p.shape) for p in pyr] == [(14080, 1, 55, 128), (14080, 1, 27, 64), (14080, 1, 13, 32), (14080, 1, 6, 16)]
    tp = torch.ops.oflow.corr_pyramid_tiled(f, f, 4)
    per = [int(_native.load().oflow_corr_tiled_level_floats(h, w)) for h, w in _native.pyramid_dims(55, 128, 4)]
    assert [tuple(t.shape) for t in tp] == [(14080, n) for n in per]
    co = torch.empty(2, 2, 55, 128, device=META)
    assert tuple(torch.ops.oflow.corr_lookup(pyr, co, 4).shape) == (2, 324, 55, 128)
    assert tuple(torch.ops.oflow.corr_lookup_tiled(tp, co, 3).shape) == (2, 196, 55, 128)
    f1h, f2h = torch.ops.oflow.corr_otf_prepare(f, f, 3)
    assert f1h.dtype == torch.float16 and tuple(f1h.shape) == (2, 55, 128, 64)
    assert [tuple(t.shape) for t in f2h] == [(2, 55, 128, 64), (2, 27, 64, 64), (2, 13, 32, 64)]
    assert tuple(torch.ops.oflow.corr_lookup_otf(f1h, f2h, co, 4).shape) == (2, 243, 55, 128)
    fr = torch.empty(3, 5, 20, 30, device=META)
    assert tuple(torch.ops.oflow.grid_warp(fr, torch.empty(3, 2, 20, 30, device=META), 0, 1, False).shape) == (3, 5, 20, 30)
    assert tuple(torch.ops.oflow.grid_sample(fr, torch.empty(3, 7, 9, 2, device=META), 2, 0, True).shape) == (3, 5, 7, 9)


def test_meta_argument_checks():
    _native.load()
    f = torch.empty(1, 64, 16, 16, device=META)
    co = torch.empty(1, 2, 16, 16, device=META)
    pyr = torch.ops.oflow.corr_pyramid(f, f, 2)
    with pytest.raises(RuntimeError, match="radius 8 outside"):
        torch.ops.oflow.corr_lookup(pyr, co, 8)
    with pytest.raises(RuntimeError, match="must be equal"):
        torch.ops.oflow.corr_pyramid(f, torch.empty(1, 64, 16, 8, device=META), 2)
    with pytest.raises(RuntimeError, match="C % 32"):
        torch.ops.oflow.corr_otf_prepare(torch.empty(1, 40, 16, 16, device=META), torch.empty(1, 40, 16, 16, device=META), 2)
    with pytest.raises(ValueError, match="interpolation mode"):
        torch.ops.oflow.grid_warp(torch.empty(1, 3, 4, 4, device=META), torch.empty(1, 2, 4, 4, device=META), 5, 0, False)


def test_autograd_formulas_are_wired():
    """Gradients flow (as shapes, on meta tensors) through pyramid -> lookup and through warp / grid_sample."""
    _native.load()
    f1 = torch.empty(2, 32, 16, 16, device=META, requires_grad=True)
    f2 = torch.empty(2, 32, 16, 16, device=META, requires_grad=True)
    pyr = _native.corr_pyramid(f1, f2, 3)
    out = _native.corr_lookup(pyr, torch.empty(2, 2, 16, 16, device=META), 2)
    assert out.requires_grad
    out.sum().backward()
    assert f1.grad.shape == f1.shape and f2.grad.shape == f2.shape
    fr = torch.empty(1, 3, 8, 8, device=META, requires_grad=True)
    fl = torch.empty(1, 2, 8, 8, device=META, requires_grad=True)
    _native.grid_warp(fr, fl, "bicubic", "zeros", True).sum().backward()
    assert fr.grad.shape == fr.shape and fl.grad.shape == fl.shape
    g = torch.empty(1, 5, 6, 2, device=META, requires_grad=True)
    _native.grid_sample(fr.detach().requires_grad_(), g, "bilinear", "zeros", True).sum().backward()
    assert g.grad.shape == g.shape


def test_cpu_tensors_raise():
    _native.load()
    x = torch.zeros(1, 8, 16, 16)
    for call in (
        lambda: torch.ops.oflow.corr_pyramid(x, x, 2),
        lambda: torch.ops.oflow.corr_pyramid_tiled(x, x, 2),
        lambda: torch.ops.oflow.corr_lookup([torch.zeros(256, 1, 16, 16)], torch.zeros(1, 2, 16, 16), 2),
        lambda: torch.ops.oflow.grid_warp(torch.zeros(1, 3, 4, 4), torch.zeros(1, 2, 4, 4), 0, 0, False),
        lambda: torch.ops.oflow.grid_sample(torch.zeros(1, 3, 4, 4), torch.zeros(1, 2, 2, 2), 0, 0, False),
        lambda: torch.ops.oflow.corr_otf_prepare(torch.zeros(1, 32, 8, 8), torch.zeros(1, 32, 8, 8), 1),
    ):
        with pytest.raises(RuntimeError, match="no CPU fallback"):
            call()
