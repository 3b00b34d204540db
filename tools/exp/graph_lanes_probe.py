"""Two-lane GraphedRAFT capture probe (r05; the r04 two-lane capture segfaulted in capture_end,
profiles/r04/s12_graph8.log). One configuration per process, selected by VARIANT:
    flag      -- this tree: capture_active() flag around the capture (weight caches never wait on pre-capture events)
    initmain  -- flag + RAFT.lane_init_on_main (lane buffers allocated on the capture stream before the fork)
    noside    -- flag + no side streams inside the lanes (update_block.split_streams = False: no fork from a lane)
Before capture_end, for every persistent side / lane stream the forward used, prints whether the stream reports itself
as capturing (torch.cuda.is_current_stream_capturing under that stream). Then replays and compares with the eager
two-lane forward bit for bit, and times both. Prints one JSON line.
    VARIANT=flag PAIRS=8 python -X faulthandler tools/exp/graph_lanes_probe.py"""
import json
import os
import statistics
import sys

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
for p in (REPO, os.path.join(REPO, "torch-optical-flow_amd"), os.path.join(REPO, "torch-optical-flow_amd", "methods", "raft")):
    sys.path.insert(0, p)

import torch  # noqa: E402

from model import RAFT, InputPadder, synthetic  # noqa: E402
from model import graph as G  # noqa: E402
from model import update as U  # noqa: E402


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
    variant = os.environ.get("VARIANT", "flag")
    pairs = int(os.environ.get("PAIRS", "8"))
    dev = torch.device("cuda", 0)
    model = RAFT().eval()
    model.load_state_dict(synthetic.synthetic_state_dict(model.state_dict()))
    model = model.to(dev)
    model.pair_lanes = 2
    G.CAPTURE_LANE_SIDE_STREAMS = None  # capture exactly as configured below
    model.lane_init_on_main = variant == "initmain"
    if variant == "noside":
        model.update_block.split_streams = False
    a0, a1 = synthetic.synthetic_pair(2, 436, 1024, seed=0)
    padder = InputPadder((436, 1024), mode="sintel")
    reps = -(-pairs // 2)
    p0, p1 = padder.pad(a0.to(dev).repeat(reps, 1, 1, 1)[:pairs], a1.to(dev).repeat(reps, 1, 1, 1)[:pairs])
    out = {"variant": variant, "pairs": pairs}

    # report the capture status of every persistent stream just before capture_end
    real_forward = model._forward
    status = {}

    def probed_forward(*a, **k):
        r = real_forward(*a, **k)
        if torch.cuda.is_current_stream_capturing():
            for key, st in U._SIDE_STREAMS.items():
                with torch.cuda.stream(st):
                    status[str(key)] = bool(torch.cuda.is_current_stream_capturing())
        return r

    model._forward = probed_forward
    with torch.inference_mode():
        ref = model(p0, p1, iters=12, test_mode=True)[1].clone()
        print("eager ok", flush=True)
        g = G.GraphedRAFT(model, p0, p1, iters=12)
        print("captured; stream capture status:", json.dumps(status), flush=True)
        up = g(p0, p1)[1].clone()
        torch.cuda.synchronize()
        out["stream_capturing"] = status
        out["bit_identical"] = bool(torch.equal(up, ref))
        out["max_abs_diff"] = (up - ref).abs().max().item()
        # new inputs: the replay follows them
        q0, q1 = p1.clone(), p0.clone()
        ref2 = model(q0, q1, iters=12, test_mode=True)[1].clone()
        up2 = g(q0, q1)[1].clone()
        out["bit_identical_new_inputs"] = bool(torch.equal(up2, ref2))
        out["graph_ms"] = timed(lambda: g(p0, p1))
        out["eager_2lanes_ms"] = timed(lambda: model(p0, p1, iters=12, test_mode=True))
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
