"""Probe GraphedRAFT at a batch / lane setting (one configuration per process): capture, replay, compare with the
eager forward, time both. PAIRS, LANES env. Prints one JSON line.
    PAIRS=8 LANES=1 python tools/exp/graph_probe.py"""
import json
import os
import statistics
import sys

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
for p in (REPO, os.path.join(REPO, "torch-optical-flow_amd"), os.path.join(REPO, "torch-optical-flow_amd", "methods", "raft")):
    sys.path.insert(0, p)

import torch  # noqa: E402

from model import RAFT, InputPadder, synthetic  # noqa: E402
from model.graph import GraphedRAFT  # noqa: E402


def timed(fn, reps=10):
    fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        b.synchronize()
        ts.append(a.elapsed_time(b))
    return round(statistics.median(ts), 3)


def main():
    pairs, lanes = int(os.environ.get("PAIRS", "8")), int(os.environ.get("LANES", "1"))
    dev = torch.device("cuda", 0)
    model = RAFT().eval()
    model.load_state_dict(synthetic.synthetic_state_dict(model.state_dict()))
    model = model.to(dev)
    model.pair_lanes = lanes
    a0, a1 = synthetic.synthetic_pair(2, 436, 1024, seed=0)
    padder = InputPadder((436, 1024), mode="sintel")
    reps = -(-pairs // 2)
    p0, p1 = padder.pad(a0.to(dev).repeat(reps, 1, 1, 1)[:pairs], a1.to(dev).repeat(reps, 1, 1, 1)[:pairs])
    out = {"pairs": pairs, "lanes": lanes}
    with torch.inference_mode():
        ref = model(p0, p1, iters=12, test_mode=True)[1].clone()
        print("eager ok", flush=True)
        g = GraphedRAFT(model, p0, p1, iters=12)
        print("captured", flush=True)
        up = g(p0, p1)[1].clone()
        torch.cuda.synchronize()
        out["max_abs_diff"] = (up - ref).abs().max().item()
        out["graph_ms"] = timed(lambda: g(p0, p1))
        model.pair_lanes = 2
        out["eager_2lanes_ms"] = timed(lambda: model(p0, p1, iters=12, test_mode=True))
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
