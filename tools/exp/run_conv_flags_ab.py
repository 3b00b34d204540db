"""In-process A/B of conv_s32 experiment flags (oflow_exp_set_conv_flags) on the RAFT Sintel x8 step (12 iterations,
test mode): FLAGS=0,512,1024,1536 (comma list); rounds interleaved, 3 forwards per sample; the flows of every setting
compared bit for bit with the first. Prints one JSON line."""
import ctypes
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
    flags = [int(v) for v in os.environ.get("FLAGS", "0,512").split(",")]
    lib = N.load()
    lib.oflow_exp_set_conv_flags.argtypes = [ctypes.c_int]
    dev = torch.device("cuda", 0)
    model = RAFT().eval()
    model.load_state_dict(synthetic.synthetic_state_dict(model.state_dict()))
    model = model.to(dev)
    a0, a1 = synthetic.synthetic_pair(2, 436, 1024, seed=0)
    padder = InputPadder((436, 1024), mode="sintel")
    p0, p1 = padder.pad(a0.to(dev).repeat(4, 1, 1, 1), a1.to(dev).repeat(4, 1, 1, 1))
    res, ref, same = {f: [] for f in flags}, None, {}
    with torch.inference_mode():
        for f in flags:
            lib.oflow_exp_set_conv_flags(f)
            up = model(p0, p1, iters=12, test_mode=True)[1].clone()
            if ref is None:
                ref = up
            same[f] = bool(torch.equal(up, ref))
        for _ in range(int(os.environ.get("ROUNDS", "5"))):
            for f in flags:
                lib.oflow_exp_set_conv_flags(f)
                model(p0, p1, iters=12, test_mode=True)
                torch.cuda.synchronize()
                a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                a.record()
                for _ in range(3):
                    model(p0, p1, iters=12, test_mode=True)
                b.record()
                b.synchronize()
                res[f].append(a.elapsed_time(b) / 3)
    lib.oflow_exp_set_conv_flags(0)
    print(json.dumps({"ms_per_step": {str(f): {"median": round(statistics.median(v), 3), "min": round(min(v), 3)}
                                      for f, v in res.items()}, "bit_identical": {str(k): v for k, v in same.items()}}))


if __name__ == "__main__":
    main()
