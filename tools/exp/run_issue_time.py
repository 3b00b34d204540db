"""EXPERIMENT: host issue time vs. GPU time of one RAFT Sintel x8 forward (is the step launch-bound?)."""
import os
import statistics
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
PKG = os.path.join(REPO, "torch-optical-flow_amd")
for p in (REPO, PKG, os.path.join(PKG, "methods", "raft")):
    sys.path.insert(0, p)

import torch  # noqa: E402

from model import RAFT, InputPadder, synthetic  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    model = RAFT().eval()
    model.load_state_dict(synthetic.synthetic_state_dict(model.state_dict()))
    model = model.to(dev)
    a0, a1 = synthetic.synthetic_pair(2, 436, 1024, seed=0)
    p0, p1 = InputPadder((436, 1024), mode="sintel").pad(a0.to(dev).repeat(4, 1, 1, 1), a1.to(dev).repeat(4, 1, 1, 1))
    with torch.inference_mode():
        for lanes in (1, 2):
            model.pair_lanes = lanes
            for _ in range(2):
                model(p0, p1, iters=12, test_mode=True)
            issue, total = [], []
            for _ in range(8):
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                model(p0, p1, iters=12, test_mode=True)
                t1 = time.perf_counter()
                torch.cuda.synchronize()
                t2 = time.perf_counter()
                issue.append((t1 - t0) * 1e3)
                total.append((t2 - t0) * 1e3)
            print(f"lanes={lanes}: host issue {statistics.median(issue):.2f} ms, issue+drain {statistics.median(total):.2f} ms",
                  flush=True)


if __name__ == "__main__":
    main()
