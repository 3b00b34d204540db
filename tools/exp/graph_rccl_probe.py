"""Capture GraphedRAFT while an RCCL communicator is live (bench.py --gpus N runs that way): world size 1 over the nccl
backend (127.0.0.1), one all_reduce to instantiate the communicator and its proxy thread, then capture (capture error
mode given by GRAPH_CAPTURE_MODE, default the model's) and replay 3 times; the flows must equal the eager forward's.
Prints one JSON line."""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
for p in (REPO, os.path.join(REPO, "torch-optical-flow_amd"), os.path.join(REPO, "torch-optical-flow_amd", "methods", "raft")):
    sys.path.insert(0, p)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from model import RAFT, InputPadder, synthetic  # noqa: E402
from model.graph import GraphedRAFT  # noqa: E402


def main():
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29531")
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    t = torch.ones(4, device=dev)
    dist.all_reduce(t)
    torch.cuda.synchronize()
    model = RAFT().eval()
    model.load_state_dict(synthetic.synthetic_state_dict(model.state_dict()))
    model = model.to(dev)
    a0, a1 = synthetic.synthetic_pair(2, 436, 1024, seed=0)
    padder = InputPadder((436, 1024), mode="sintel")
    p0, p1 = padder.pad(a0.to(dev).repeat(2, 1, 1, 1), a1.to(dev).repeat(2, 1, 1, 1))
    out = {}
    with torch.inference_mode():
        lo_e, up_e = model(p0, p1, iters=12, test_mode=True)
        g = GraphedRAFT(model, p0, p1, iters=12)
        for i in range(3):
            dist.all_reduce(t)  # the communicator stays busy between replays
            lo, up = g(p0, p1)
        torch.cuda.synchronize()
        out["equal"] = bool(torch.equal(lo, lo_e) and torch.equal(up, up_e))
    out["all_reduce"] = float(t[0])
    dist.destroy_process_group()
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
