"""EXPERIMENT: RAFT Sintel x8 forward with different output-channel blocks for the update-block convs
(model.update.CONV_BN), interleaved in one process. Results must be bit-identical (same k order per output)."""
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
from model import update as U  # noqa: E402


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
    base = dict(U.CONV_BN)
    cfgs = {"base": {}, "c2=96": {"c2": 96}, "f2=32": {"f2": 32}, "fh1=64": {"fh1": 64}, "mo=64": {"mo": 64}}
    res = {k: [] for k in cfgs}
    outs = {}

    def setf(k):
        U.CONV_BN.clear()
        U.CONV_BN.update(base)
        U.CONV_BN.update(cfgs[k])

    with torch.inference_mode():
        for k in cfgs:
            setf(k)
            outs[k] = model(p0, p1, iters=12, test_mode=True)[1].clone()
        torch.cuda.synchronize()
        for k in cfgs:
            print(f"{k}: identical to base: {bool(torch.equal(outs[k], outs['base']))}", flush=True)
        for _ in range(5):
            for k in cfgs:
                setf(k)
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
