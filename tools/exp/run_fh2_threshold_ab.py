"""EXPERIMENT: RAFT Sintel x8 forward (two 4-pair lanes of 28160 px) with the flow head's output conv as
oflow_conv_s32 (default above 16384 px) vs oflow_flow_head2_s32 (fp32 FMAs), interleaved in one process."""
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
from optical_flow import _native  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    model = RAFT().eval()
    model.load_state_dict(synthetic.synthetic_state_dict(model.state_dict()))
    model = model.to(dev)
    a0, a1 = synthetic.synthetic_pair(2, 436, 1024, seed=0)
    img0 = a0.to(dev).repeat(4, 1, 1, 1)
    img1 = a1.to(dev).repeat(4, 1, 1, 1)
    padder = InputPadder((436, 1024), mode="sintel")
    p0, p1 = padder.pad(img0, img1)
    cfgs = {"conv_s32 (default)": 16384, "flow_head2 FMA": 1 << 30}
    res = {k: [] for k in cfgs}
    outs = {}
    with torch.inference_mode():
        for k, v in cfgs.items():
            _native.FLOW_HEAD2_MAX_PIXELS = v
            outs[k] = model(p0, p1, iters=12, test_mode=True)[1].clone()
        torch.cuda.synchronize()
        d = (outs["flow_head2 FMA"] - outs["conv_s32 (default)"]).abs()
        print(f"max |flow difference| {float(d.max()):.3e} px, mean {float(d.mean()):.3e}", flush=True)
        for _ in range(6):
            for k, v in cfgs.items():
                _native.FLOW_HEAD2_MAX_PIXELS = v
                a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                a.record()
                for _ in range(3):
                    model(p0, p1, iters=12, test_mode=True)
                b.record()
                b.synchronize()
                res[k].append(a.elapsed_time(b) / 3)
    for k, v in res.items():
        print(f"{k}: median {statistics.median(v):.3f} ms/step, min {min(v):.3f}", flush=True)


if __name__ == "__main__":
    main()
