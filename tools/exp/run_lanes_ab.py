"""EXPERIMENT: RAFT Sintel x8 forward with the update loop on one stream vs. 2-4 pair lanes (joined / per-lane lookup),
interleaved in one process. Results: profiles/r01/exp/pair_lanes_ab.log (runs 2-3 on another box; run 3 with
GPU_MAX_HW_QUEUES=8)."""
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


def main():
    dev = torch.device("cuda", 0)
    torch.backends.cudnn.benchmark = True
    model = RAFT().eval()
    model.load_state_dict(synthetic.synthetic_state_dict(model.state_dict()))
    model = model.to(dev)
    a0, a1 = synthetic.synthetic_pair(2, 436, 1024, seed=0)
    img0 = a0.to(dev).repeat(4, 1, 1, 1)
    img1 = a1.to(dev).repeat(4, 1, 1, 1)
    padder = InputPadder((436, 1024), mode="sintel")
    p0, p1 = padder.pad(img0, img1)
    cfgs = {"1 lane": (1, "joined"), "2 lanes joined": (2, "joined"), "2 lanes own lookup": (2, "lane"),
            "3 lanes joined": (3, "joined"), "4 lanes joined": (4, "joined"), "4 lanes own lookup": (4, "lane")}
    res = {k: [] for k in cfgs}

    def setf(k):
        model.pair_lanes, model.pair_lookup = cfgs[k]

    with torch.inference_mode():
        for k in cfgs:
            setf(k)
            model(p0, p1, iters=12, test_mode=True)
        torch.cuda.synchronize()
        outs = {}
        for k in cfgs:
            setf(k)
            outs[k] = model(p0, p1, iters=12, test_mode=True)[1].clone()
        torch.cuda.synchronize()
        print("outputs equal across lane configs:", all(torch.equal(outs[k], outs["1 lane"]) for k in cfgs), flush=True)
        for _ in range(6):
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
