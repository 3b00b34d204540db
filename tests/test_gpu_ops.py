"""``torch.ops.oflow`` on the GPU: the ops equal the C-ABI path they wrap, and CorrBlock.__call__ + warp compile with
``torch.compile(fullgraph=True)`` (no graph breaks) to the same values as eager."""
import pytest
import torch

import optical_flow
from model import CorrBlock, synthetic
from model.utils import coords_grid
from optical_flow import _native

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)


def _inputs(b=2, c=64, h=24, w=40, seed=5):
    f1, f2 = synthetic.synthetic_fmaps(b, c, h, w, stream=seed)
    coords = coords_grid(b, h, w) + torch.from_numpy(synthetic.hash_normal(seed, (b, 2, h, w), 3.0))
    return f1.to(DEV), f2.to(DEV), coords.to(DEV)


def test_ops_equal_c_abi_path():
    f1, f2, coords = _inputs()
    cb = CorrBlock(f1, f2)
    a = cb(coords)
    b = torch.ops.oflow.corr_lookup_tiled(cb._tiled.levels, coords, 4)
    c = torch.ops.oflow.corr_lookup(torch.ops.oflow.corr_pyramid(f1, f2, 4), coords, 4)
    assert torch.equal(a, b) and torch.equal(a, c)


def test_compile_fullgraph_corrblock_and_warp():
    torch._dynamo.reset()
    f1, f2, coords = _inputs()
    with torch.no_grad():
        cb = CorrBlock(f1, f2)
        frame = torch.rand(2, 3, 24, 40, device=DEV)
        flow = optical_flow.normalize(coords - coords_grid(2, 24, 40, device=DEV))

        def step(coords, frame, flow):
            return cb(coords), optical_flow.warp(frame, flow)

        eager = step(coords, frame, flow)
        compiled = torch.compile(step, fullgraph=True, dynamic=False)
        got = compiled(coords, frame, flow)
        got2 = compiled(coords + 0.25, frame, flow)
    assert torch.equal(got[0], eager[0]) and torch.equal(got[1], eager[1])
    assert torch.equal(got2[0], cb(coords + 0.25))


def test_compile_fullgraph_training_lookup():
    """The canonical (autograd) pyramid + lookup traced as one graph, backward included."""
    torch._dynamo.reset()
    f1, f2, coords = _inputs(b=1, c=32, h=16, w=16)

    def loss(a, b, co):
        pyr = torch.ops.oflow.corr_pyramid(a, b, 3)
        return torch.ops.oflow.corr_lookup(pyr, co, 2).square().sum()

    grads = []
    for fn in (loss, torch.compile(loss, fullgraph=True, dynamic=False)):
        a, b = f1.clone().requires_grad_(), f2.clone().requires_grad_()
        fn(a, b, coords).backward()
        grads.append((a.grad, b.grad))
    torch.testing.assert_close(grads[1][0], grads[0][0], rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(grads[1][1], grads[0][1], rtol=1e-5, atol=1e-5)
