"""Host enqueue time vs GPU time of one 8-pair RAFT forward (Sintel, 12 iterations): the forward called after a device
sync (empty queues) -- host time = until the call returns; GPU time = until the device is idle. Counts kernel launches
through the native layer. Prints one JSON line."""
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
for p in (REPO, os.path.join(REPO, "torch-optical-flow_amd"), os.path.join(REPO, "torch-optical-flow_amd", "methods", "raft")):
    sys.path.insert(0, p)

import torch  # noqa: E402

from model import RAFT, InputPadder, synthetic  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    model = RAFT().eval()
    model.load_state_dict(synthetic.synthetic_state_dict(model.state_dict()))
    model = model.to(dev)
    pairs = int(os.environ.get("PAIRS", "8"))
    a0, a1 = synthetic.synthetic_pair(pairs, 436, 1024, seed=0)
    padder = InputPadder((436, 1024), mode="sintel")
    p0, p1 = padder.pad(a0.to(dev), a1.to(dev))
    out = {}
    with torch.inference_mode():
        for _ in range(3):
            model(p0, p1, iters=12, test_mode=True)
        torch.cuda.synchronize()
        hs, gs = [], []
        for _ in range(5):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            model(p0, p1, iters=12, test_mode=True)
            t1 = time.perf_counter()
            torch.cuda.synchronize()
            t2 = time.perf_counter()
            hs.append((t1 - t0) * 1e3)
            gs.append((t2 - t0) * 1e3)
        out["host_enqueue_ms"] = round(min(hs), 3)
        out["forward_ms"] = round(min(gs), 3)
        # back-to-back forwards (the bench's regime)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(10):
            model(p0, p1, iters=12, test_mode=True)
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        out["b2b_host_ms_per_forward"] = round((t1 - t0) * 1e2, 3)
        out["b2b_ms_per_forward"] = round((t2 - t0) * 1e2, 3)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
