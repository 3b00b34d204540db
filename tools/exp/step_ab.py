"""RAFT Sintel x8 forward (12 iterations, test mode) ms/step in this process's build (OFLOW_LIB / OFLOW_OPS_LIB select
another one, tools/build_rev.sh): 3 forwards per sample, 6 samples after a warm-up. Back-to-back processes with
different libraries give the A/B. Prints one JSON line."""
import json
import os
import statistics
import sys

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
for p in (REPO, os.path.join(REPO, "torch-optical-flow_amd"), os.path.join(REPO, "torch-optical-flow_amd", "methods", "raft")):
    sys.path.insert(0, p)

import torch  # noqa: E402

from optical_flow import _native as N  # noqa: E402
from model import RAFT, InputPadder, synthetic  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    model = RAFT().eval()
    model.load_state_dict(synthetic.synthetic_state_dict(model.state_dict()))
    model = model.to(dev)
    a0, a1 = synthetic.synthetic_pair(2, 436, 1024, seed=0)
    padder = InputPadder((436, 1024), mode="sintel")
    p0, p1 = padder.pad(a0.to(dev).repeat(4, 1, 1, 1), a1.to(dev).repeat(4, 1, 1, 1))
    ts = []
    with torch.inference_mode():
        for _ in range(2):
            model(p0, p1, iters=12, test_mode=True)
        torch.cuda.synchronize()
        for _ in range(int(os.environ.get("SAMPLES", "6"))):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            for _ in range(3):
                model(p0, p1, iters=12, test_mode=True)
            b.record()
            b.synchronize()
            ts.append(a.elapsed_time(b) / 3)
    print(json.dumps({"lib": N.library_path(), "ms_per_step_median": round(statistics.median(ts), 3),
                      "ms_per_step_min": round(min(ts), 3)}), flush=True)


if __name__ == "__main__":
    main()
