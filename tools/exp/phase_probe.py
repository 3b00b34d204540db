"""Un-profiled phase split of the 8-pair Sintel forward: back-to-back forwards at 1, 2, 7 and 12 GRU iterations
(test mode); the per-iteration cost is the slope, the encoders + pyramid (+ one upsampling) the intercept. Profilers
slow the host enough to reorder the encoder streams' start, so this is the phase measurement without one."""
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
    a0, a1 = synthetic.synthetic_pair(8, 436, 1024, seed=0)
    padder = InputPadder((436, 1024), mode="sintel")
    p0, p1 = padder.pad(a0.to(dev), a1.to(dev))
    res = {}
    with torch.inference_mode():
        for it in (1, 2, 7, 12):
            for _ in range(2):
                model(p0, p1, iters=it, test_mode=True)
        for rnd in range(3):
            for it in (1, 2, 7, 12):
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                for _ in range(8):
                    model(p0, p1, iters=it, test_mode=True)
                torch.cuda.synchronize()
                res.setdefault(it, []).append((time.perf_counter() - t0) / 8 * 1e3)
    ms = {it: min(v) for it, v in res.items()}
    slope = (ms[12] - ms[2]) / 10
    out = {"ms_per_forward": {str(k): round(v, 3) for k, v in ms.items()}, "ms_per_iteration": round(slope, 3),
           "encoders_pyramid_ms": round(ms[1] - slope, 3)}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
