"""Generate the golden fixtures in tests/golden/ by running the REFERENCE itself (CPU, fp32).

Runs only in the build container, where /root/reference exists; exits 0 with a message elsewhere.
The reference is imported by file path: its ``model`` package needs
``pytorch_lightning``/``wandb``/``torchmetrics`` at import time only, so minimal stand-in modules are
registered for those three names (they add no arithmetic: ``LightningModule`` is ``nn.Module`` plus
``hparams``). Nothing from the reference is copied into the repository; only input/output arrays are
written. Bytecode writing is disabled so the read-only tree stays untouched.

Inputs come from the repository's own deterministic generators (``model/synthetic.py``), which the GPU box
re-runs bit-for-bit; fmaps are therefore not stored, only a float64 checksum that the tests re-verify.

Usage:  python tests/golden/gen_goldens.py [corr] [warp] [raft] [batch] [io] [hd]   (default: all)
"""
from __future__ import annotations

import importlib.util
import os
import sys
import types

sys.dont_write_bytecode = True
os.environ["PYTHONDONTWRITEBYTECODE"] = "1"

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.nn as nn  # noqa: E402

REF = "/root/reference"
HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))


def _load_by_path(name: str, path: str):
    spec = importlib.util.spec_from_file_location(name, path)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


synthetic = _load_by_path(
    "oflow_synthetic", os.path.join(REPO, "torch-optical-flow_amd", "methods", "raft", "model", "synthetic.py")
)


def _install_stubs() -> None:
    class _HParams(dict):
        def __getattr__(self, k):
            try:
                return self[k]
            except KeyError as e:  # copy.deepcopy probes attributes; must be AttributeError
                raise AttributeError(k) from e

    class LightningModule(nn.Module):
        def save_hyperparameters(self):
            frame = sys._getframe(1)
            args = {k: v for k, v in frame.f_locals.items() if k not in ("self", "__class__")}
            self.hparams = _HParams(args)

    pl = types.ModuleType("pytorch_lightning")
    pl.LightningModule = LightningModule
    pl_loggers = types.ModuleType("pytorch_lightning.loggers")
    pl_loggers.WandbLogger = type("WandbLogger", (), {})
    pl.loggers = pl_loggers
    wandb = types.ModuleType("wandb")
    wandb.Image = type("Image", (), {})

    class Metric(nn.Module):
        def add_state(self, name, default, dist_reduce_fx=None):
            setattr(self, name, default)

    tm = types.ModuleType("torchmetrics")
    tm.Metric = Metric
    for name, mod in {
        "pytorch_lightning": pl,
        "pytorch_lightning.loggers": pl_loggers,
        "wandb": wandb,
        "torchmetrics": tm,
    }.items():
        sys.modules.setdefault(name, mod)


def _import_reference():
    _install_stubs()
    sys.path[:0] = [os.path.join(REF, "methods", "raft"), REF]
    import optical_flow  # noqa: F401  (reference package; needs the torchmetrics stand-in)
    from model import RAFT  # reference methods/raft/model
    from model.corr import CorrBlock
    from model.utils import InputPadder, bilinear_sampler, coords_grid
    from optical_flow.operator import operator as ref_operator

    return RAFT, CorrBlock, InputPadder, bilinear_sampler, coords_grid, ref_operator


def _checksum(t: torch.Tensor) -> np.ndarray:
    a = t.detach().double().numpy()
    return np.array([a.sum(), (a * a).sum(), np.abs(a).max()], dtype=np.float64)


def gen_corr(CorrBlock, coords_grid) -> None:
    """CorrBlock build + lookup (`corr.py:38-87`, `utils.py:64-86`)."""
    cases = {"a": (1, 16, 20, 7), "b": (2, 16, 17, 11)}
    out = {}
    for tag, (B, H, W, stream) in cases.items():
        f1, f2 = synthetic.synthetic_fmaps(B, 256, H, W, stream=stream)
        out[f"{tag}_shape"] = np.array([B, 256, H, W], dtype=np.int64)
        out[f"{tag}_stream"] = np.array(stream, dtype=np.int64)
        out[f"{tag}_fmap1_checksum"] = _checksum(f1)
        out[f"{tag}_fmap2_checksum"] = _checksum(f2)
        cb = CorrBlock(f1, f2, num_levels=4, radius=4)
        for lvl, p in enumerate(cb.corr_pyramid):
            out[f"{tag}_pyr{lvl}"] = p.numpy()
        base = coords_grid(B, H, W)
        sigmas = (0.0, 3.0, 20.0) if tag == "a" else (3.0,)
        for k, sigma in enumerate(sigmas):
            noise = torch.from_numpy(synthetic.hash_normal(500 + 10 * stream + k, base.shape, sigma))
            coords = base + noise
            out[f"{tag}_coords_s{int(sigma)}"] = coords.numpy()
            out[f"{tag}_lookup_s{int(sigma)}"] = cb(coords).numpy()
        if tag == "a":
            # coords exactly on the last valid column/row of every level and beyond (Q4 boundary)
            edge = base.clone()
            edge[:, 0] = float(W - 1)
            edge[:, 1] = torch.linspace(-2.0, float(H + 1), H)[None, :, None].expand(B, H, W)
            out["a_coords_edge"] = edge.numpy()
            out["a_lookup_edge"] = cb(edge).numpy()
            # radius 2 / 3 levels (non-default CorrBlock arguments, `corr.py:38-40`)
            cb2 = CorrBlock(f1, f2, num_levels=3, radius=2)
            c3 = base + torch.from_numpy(synthetic.hash_normal(777, base.shape, 2.0))
            out["a_coords_r2"] = c3.numpy()
            out["a_lookup_r2_l3"] = cb2(c3).numpy()
    np.savez_compressed(os.path.join(HERE, "corr_small.npz"), **out)


def gen_warp(ref_operator) -> None:
    """``warp`` / ``grid_sample`` in every mode (`operator.py:8-56`)."""
    B, C, H, W = 2, 3, 13, 17
    frame = torch.from_numpy((synthetic.hash_uniform(900, B * C * H * W) * 255.0).astype(np.float32)).view(B, C, H, W)
    flow_px = torch.from_numpy(synthetic.hash_normal(901, (B, 2, H, W), 3.0))
    flow_px[0, :, 0, :4] = torch.tensor([[40.0, -40.0, 0.5, 8.0], [0.0, 3.0, -30.0, 15.0]])
    flow = ref_operator.normalize(flow_px)
    out = {"frame": frame.numpy(), "flow": flow.numpy(), "flow_px": flow_px.numpy()}
    for mode in ("bilinear", "nearest", "bicubic"):
        for pad in ("zeros", "border", "reflection"):
            for ac in (False, True):
                out[f"warp_{mode}_{pad}_{int(ac)}"] = ref_operator.warp(frame, flow, mode, pad, ac).numpy()
    out["warp_default"] = ref_operator.warp(frame, flow).numpy()
    out["grid"] = ref_operator.warp_grid(flow.permute(0, 2, 3, 1)).numpy()
    out["integrate_3"] = ref_operator.integrate(flow_px, 0.5 * flow_px, -0.25 * flow_px).numpy()
    np.savez_compressed(os.path.join(HERE, "warp_small.npz"), **out)


def gen_raft(RAFT, InputPadder) -> None:
    """RAFT forward(test_mode=True) with predict.py's padding (`raft.py:87-147`, `predict.py:84-89`)."""
    torch.set_num_threads(max(1, os.cpu_count() or 1))
    model = RAFT()
    model.load_state_dict(synthetic.synthetic_state_dict(model.state_dict()))
    model.eval()
    cases = {
        "sintel": dict(B=1, H=436, W=1024, iters=12, stride=4, mode="sintel", seed=0),
        "small": dict(B=1, H=128, W=128, iters=12, stride=1, mode="sintel", seed=3),
        "small24": dict(B=1, H=128, W=128, iters=24, stride=1, mode="sintel", seed=3),
        "kitti": dict(B=2, H=375, W=1242, iters=12, stride=4, mode="sintel", seed=5),
        "kittimode": dict(B=1, H=150, W=203, iters=6, stride=1, mode="kitti", seed=9),
    }
    out = {}
    with torch.inference_mode():
        for tag, c in cases.items():
            img0, img1 = synthetic.synthetic_pair(c["B"], c["H"], c["W"], seed=c["seed"])
            padder = InputPadder(img0.shape, mode=c["mode"])
            p0, p1 = padder.pad(img0, img1)
            low, up = model(p0, p1, iters=c["iters"], test_mode=True)
            up = padder.unpad(up)
            s = c["stride"]
            out[f"{tag}_cfg"] = np.array([c["B"], c["H"], c["W"], c["iters"], s, c["seed"]], dtype=np.int64)
            out[f"{tag}_mode"] = np.array(c["mode"])
            out[f"{tag}_low"] = low.numpy()
            out[f"{tag}_up"] = up[..., ::s, ::s].contiguous().numpy()
            out[f"{tag}_up_checksum"] = _checksum(up)
            print(tag, "flow_up mean |f| =", float(up.norm(dim=1).mean()), flush=True)
    np.savez_compressed(os.path.join(HERE, "raft_e2e.npz"), **out)


BATCH_CASES = {
    # the benchmarked configurations themselves (bench.py WORKLOADS "sintel" / "kitti": 8 pairs per GPU, 12 iters,
    # 'sintel' padding): at 8 pairs the update loop runs on two pair lanes and the flow head's output conv on the
    # split MFMA kernel (above FLOW_HEAD2_MAX_PIXELS), the path the bench times
    "sintel8": dict(B=8, H=436, W=1024, iters=12, stride=8, mode="sintel", seed=0),
    "kitti8": dict(B=8, H=375, W=1242, iters=12, stride=8, mode="sintel", seed=5),
}


def gen_raft_batch(RAFT, InputPadder) -> None:
    """RAFT forward(test_mode=True) at the benchmarked batch (`raft.py:87-147`), written to raft_e2e_batch.npz: the
    full 1/8-res flow and the full-res flow at stride 8, per pair."""
    torch.set_num_threads(max(1, os.cpu_count() or 1))
    model = RAFT()
    model.load_state_dict(synthetic.synthetic_state_dict(model.state_dict()))
    model.eval()
    out = {}
    with torch.inference_mode():
        for tag, c in BATCH_CASES.items():
            img0, img1 = synthetic.synthetic_pair(c["B"], c["H"], c["W"], seed=c["seed"])
            padder = InputPadder(img0.shape, mode=c["mode"])
            p0, p1 = padder.pad(img0, img1)
            low, up = model(p0, p1, iters=c["iters"], test_mode=True)
            up = padder.unpad(up)
            s = c["stride"]
            out[f"{tag}_cfg"] = np.array([c["B"], c["H"], c["W"], c["iters"], s, c["seed"]], dtype=np.int64)
            out[f"{tag}_mode"] = np.array(c["mode"])
            out[f"{tag}_low"] = low.numpy()
            out[f"{tag}_up"] = up[..., ::s, ::s].contiguous().numpy()
            out[f"{tag}_up_checksum"] = _checksum(up)
            out[f"{tag}_img_checksum"] = np.stack([_checksum(img0), _checksum(img1)])
            print(tag, "flow_up mean |f| =", float(up.norm(dim=1).mean()), flush=True)
    np.savez_compressed(os.path.join(HERE, "raft_e2e_batch.npz"), **out)


HD_CASES = {
    # BASELINE configs[4]: one 1080x1920 pair, 12 iterations, 'sintel' padding (1088x1920). The reference's alternate
    # corr needs its alt_cuda_corr CUDA extension (absent, and not runnable on CPU), so the golden is the reference's
    # dense fp32 CPU path: the same correlation values (corr.py:38-87 vs the AlternateCorrBlock's definition); the GPU
    # test runs RAFT(alternate_corr=True) against it at SURVEY §8(c)'s fp16 bar.
    "hd1": dict(B=1, H=1080, W=1920, iters=12, stride=8, mode="sintel", seed=11),
}


def gen_raft_hd(RAFT, InputPadder) -> None:
    """RAFT forward(test_mode=True) at 1080p (`raft.py:87-147`), written to raft_e2e_hd.npz in raft_e2e_batch.npz's
    layout: the full 1/8-res flow, the full-res flow at stride 8, input checksums."""
    torch.set_num_threads(max(1, os.cpu_count() or 1))
    model = RAFT()
    model.load_state_dict(synthetic.synthetic_state_dict(model.state_dict()))
    model.eval()
    out = {}
    with torch.inference_mode():
        for tag, c in HD_CASES.items():
            img0, img1 = synthetic.synthetic_pair(c["B"], c["H"], c["W"], seed=c["seed"])
            padder = InputPadder(img0.shape, mode=c["mode"])
            p0, p1 = padder.pad(img0, img1)
            low, up = model(p0, p1, iters=c["iters"], test_mode=True)
            up = padder.unpad(up)
            s = c["stride"]
            out[f"{tag}_cfg"] = np.array([c["B"], c["H"], c["W"], c["iters"], s, c["seed"]], dtype=np.int64)
            out[f"{tag}_mode"] = np.array(c["mode"])
            out[f"{tag}_low"] = low.numpy()
            out[f"{tag}_up"] = up[..., ::s, ::s].contiguous().numpy()
            out[f"{tag}_up_checksum"] = _checksum(up)
            out[f"{tag}_img_checksum"] = np.stack([_checksum(img0), _checksum(img1)])
            print(tag, "flow_up mean |f| =", float(up.norm(dim=1).mean()), flush=True)
    np.savez_compressed(os.path.join(HERE, "raft_e2e_hd.npz"), **out)


def io_flows():
    """Flow fields of the I/O goldens, from the repository's own generators (the tests rebuild them)."""
    flows = {
        # the reference test's shape (tests/visualization/test_flow2rgb.py:35), hash noise instead of randn
        "n": torch.from_numpy(synthetic.hash_normal(950, (4, 2, 5, 6), 100.0)),
        "s": torch.from_numpy(synthetic.hash_normal(951, (2, 2, 37, 53), 6.0)),
    }
    # colour-wheel edges: exact axis directions (atan2 = +-pi, +-pi/2, 0: baker's k1 wrap), zero flow, one vector
    # longer than every other (rad == 1 after normalisation)
    e = torch.zeros(1, 2, 3, 4)
    e[0, :, 0, :] = torch.tensor([[-1.0, 1.0, 0.0, 0.0], [0.0, 0.0, -1.0, 1.0]])
    e[0, :, 1, :] = torch.tensor([[-5.0, 3.0, 0.25, -2.0], [1e-7, -4.0, 7.0, -2.0]])
    e[0, :, 2, 3] = torch.tensor([12.0, -9.0])
    flows["e"] = e
    return flows


IO_OPTIONS = (
    # (tag, clip, max_norm, invert_y)
    ("d", None, None, False),
    ("c1", 1.0, None, False),
    ("c50", 50.0, None, False),
    ("cpos", (0.0, 50.0), None, False),
    ("m30", None, 30.0, False),
    ("inv", None, None, True),
    ("all", 20.0, 8.0, True),
)


def gen_io() -> None:
    """flow2rgb / colorwheel (`visualization/flow2rgb.py:19-108`, `methods/*.py`) and the .flo / PFM writers
    (`io/middlebury.py:43-71`, `io/pfm.py:79-104`): expected RGB fields and file bytes."""
    from optical_flow.io.middlebury import write_middlebury
    from optical_flow.io.pfm import write_pfm
    from optical_flow.visualization.flow2rgb import colorwheel, flow2rgb

    out = {}
    for name, flow in io_flows().items():
        out[f"flow_{name}"] = flow.numpy()
        for method in ("baker", "hsv", "meister"):
            for tag, clip, max_norm, inv in IO_OPTIONS:
                if name == "e" and tag not in ("d", "inv", "m30"):
                    continue
                out[f"rgb_{name}_{method}_{tag}"] = flow2rgb(flow, method, clip, max_norm, inv).numpy()
    for method in ("baker", "hsv", "meister"):
        out[f"wheel_{method}"] = colorwheel(method, size=48).numpy()
    import tempfile

    with tempfile.TemporaryDirectory() as d:
        f = io_flows()["s"][1]
        for fmt, fn in (("flo", write_middlebury), ("pfm", write_pfm)):
            path = os.path.join(d, "x." + fmt)
            fn(path, f)
            with open(path, "rb") as fh:
                out[f"bytes_{fmt}"] = np.frombuffer(fh.read(), dtype=np.uint8)
    np.savez_compressed(os.path.join(HERE, "io_small.npz"), **out)


def main() -> int:
    if not os.path.isdir(REF):
        print("gen_goldens: /root/reference absent; fixtures are committed, nothing to do")
        return 0
    RAFT, CorrBlock, InputPadder, bilinear_sampler, coords_grid, ref_operator = _import_reference()
    which = sys.argv[1:] or ["corr", "warp", "raft", "batch", "io", "hd"]
    if "corr" in which:
        gen_corr(CorrBlock, coords_grid)
    if "warp" in which:
        gen_warp(ref_operator)
    if "raft" in which:
        gen_raft(RAFT, InputPadder)
    if "batch" in which:
        gen_raft_batch(RAFT, InputPadder)
    if "io" in which:
        gen_io()
    if "hd" in which:
        gen_raft_hd(RAFT, InputPadder)
    return 0


if __name__ == "__main__":
    sys.exit(main())
