"""Numerics experiment: does a split-precision convolution (operands as hi + lo fp16/bf16 pairs, products on
16-bit MFMA, fp32 accumulation) keep RAFT within the fp32 parity tolerance (mean EPE <= 1e-4 px)?

Runs the oracle RAFT on CPU with F.conv2d replaced by an emulation and prints the EPE against the reference's
golden flows. Emulation: x = hi + lo (each rounded to the 16-bit type), y = sum of the kept cross products,
each product exact (fp64) and the sum rounded to fp32 — an upper bound on MFMA's fp32-accumulated error.

usage: python tools/exp/split_numerics.py [small|sintel] [mode ...]
modes: fp32 (no emulation), f16x3, f16x3s (weights scaled by 2^s), f16x4, bf16x3, f16, bf16
"""
import os
import sys

import numpy as np
import torch
import torch.nn.functional as F

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [REPO, os.path.join(REPO, "torch-optical-flow_amd"), os.path.join(REPO, "torch-optical-flow_amd", "methods", "raft")]

from model import synthetic  # noqa: E402
from oracle import raft as oraft  # noqa: E402

_conv = F.conv2d


def split(x, dt, scale=1.0):
    xs = x.double() * scale
    hi = xs.to(dt).double()
    lo = (xs - hi).to(dt).double()
    return hi, lo


def make(mode):
    def conv(x, w, b=None, stride=1, padding=0, dilation=1, groups=1):
        if mode == "fp32":
            return _conv(x, w, b, stride, padding, dilation, groups)
        dt = torch.bfloat16 if mode.startswith("bf16") else torch.float16
        s = 1.0
        if mode == "f16x3s":
            s = 2.0 ** (14 - int(np.ceil(np.log2(float(w.abs().max()) + 1e-30))))
        xh, xl = split(x, dt)
        wh, wl = split(w, dt, s)
        c = lambda a, bb: _conv(a, bb, None, stride, padding, dilation, groups)  # noqa: E731
        if mode in ("f16", "bf16"):
            y = c(xh, wh)
        elif mode == "f16x4":
            y = c(xh, wh) + c(xh, wl) + c(xl, wh) + c(xl, wl)
        else:
            y = c(xh, wh) + c(xh, wl) + c(xl, wh)
        y = (y / s).float()
        if b is not None:
            y = y + b.view(1, -1, 1, 1)
        return y

    return conv


def main():
    tag = sys.argv[1] if len(sys.argv) > 1 else "small"
    modes = sys.argv[2:] or ["fp32", "f16x3", "f16x3s", "bf16x3"]
    g = np.load(os.path.join(REPO, "tests", "golden", "raft_e2e.npz"))
    b, h, w, iters, s, seed = (int(v) for v in g[f"{tag}_cfg"])
    img0, img1 = synthetic.synthetic_pair(b, h, w, seed=seed)
    padder = oraft.InputPadder(img0.shape, mode=str(g[f"{tag}_mode"]))
    p0, p1 = padder.pad(img0, img1)
    model = oraft.RAFT().eval()
    model.load_state_dict(synthetic.synthetic_state_dict(model.state_dict()))
    torch.set_num_threads(8)
    for mode in modes:
        F.conv2d = make(mode)
        torch.nn.modules.conv.F.conv2d = F.conv2d
        with torch.inference_mode():
            low, up = model(p0, p1, iters=iters, test_mode=True)
        up = padder.unpad(up)[..., ::s, ::s]
        el = torch.norm(low - torch.from_numpy(g[f"{tag}_low"]), dim=1)
        eu = torch.norm(up - torch.from_numpy(g[f"{tag}_up"]), dim=1)
        print(f"{tag} {mode:7s} low EPE mean {el.mean():.2e} max {el.max():.2e} | up mean {eu.mean():.2e} max {eu.max():.2e}", flush=True)
    F.conv2d = _conv


if __name__ == "__main__":
    main()
