"""EXPERIMENT: conv_s32 small-grid tiles (2 x 32 px, 64-channel blocks below a workgroup-count threshold) vs the default
tiles, interleaved in one process: RAFT Sintel batch 1 x 24 iterations (predict.py's case) and 8 pairs x 12."""
import ctypes
import os
import statistics
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
PKG = os.path.join(REPO, "torch-optical-flow_amd")
for p in (REPO, PKG, os.path.join(PKG, "methods", "raft")):
    sys.path.insert(0, p)

import torch  # noqa: E402

from model import RAFT, InputPadder, synthetic  # noqa: E402
from optical_flow import _native as N  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    lib = N.load()
    lib.oflow_exp_set_small_grid_px.argtypes = [ctypes.c_int]
    model = RAFT().eval()
    model.load_state_dict(synthetic.synthetic_state_dict(model.state_dict()))
    model = model.to(dev)
    a0, a1 = synthetic.synthetic_pair(2, 436, 1024, seed=0)
    padder = InputPadder((436, 1024), mode="sintel")
    cases = {"b1x24": tuple(padder.pad(a0[:1].to(dev), a1[:1].to(dev))) + (24,),
             "b8x12": tuple(padder.pad(a0.to(dev).repeat(4, 1, 1, 1), a1.to(dev).repeat(4, 1, 1, 1))) + (12,)}
    cfgs = {"default tiles": 0, "small grid < 16384 px": 16384}
    with torch.inference_mode():
        for name, (p0, p1, it) in cases.items():
            res = {k: [] for k in cfgs}
            outs = {}
            for k, v in cfgs.items():
                lib.oflow_exp_set_small_grid_px(v)
                outs[k] = model(p0, p1, iters=it, test_mode=True)[1].clone()
            torch.cuda.synchronize()
            same = all(torch.equal(outs[k], outs["default tiles"]) for k in cfgs)
            for _ in range(5):
                for k, v in cfgs.items():
                    lib.oflow_exp_set_small_grid_px(v)
                    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    a.record()
                    for _ in range(3):
                        model(p0, p1, iters=it, test_mode=True)
                    b.record()
                    b.synchronize()
                    res[k].append(a.elapsed_time(b) / 3)
            print(name, "outputs bit-identical:", same, flush=True)
            for k, v in res.items():
                print(f"  {k}: median {statistics.median(v):.3f} ms, min {min(v):.3f}", flush=True)
    lib.oflow_exp_set_small_grid_px(16384)


if __name__ == "__main__":
    main()
