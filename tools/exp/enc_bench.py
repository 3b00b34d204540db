"""Time the split encoders alone (Sintel x8 padded to 440x1024): fnet on one image batch, cnet on one, and the three
encoder streams of the RAFT forward (fnet image0 | fnet image1 | cnet image0) together. Prints one JSON line.
ARMS (optional JSON): {arm: {"<native experiment hook>": int, ...}}: the arms run interleaved in one process, each
timing taken with its hooks set (e.g. {"base": {}, "s8": {"oflow_exp_set_stats_8row": 1}}).
    python tools/exp/enc_bench.py"""
import json
import os
import statistics
import sys

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
for p in (REPO, os.path.join(REPO, "torch-optical-flow_amd"), os.path.join(REPO, "torch-optical-flow_amd", "methods", "raft")):
    sys.path.insert(0, p)

import torch  # noqa: E402

from model import RAFT, synthetic  # noqa: E402
from model.extractor import SplitEncoder  # noqa: E402


def timed(fn, reps=20):
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
    dev = torch.device("cuda", 0)
    model = RAFT().eval()
    model.load_state_dict(synthetic.synthetic_state_dict(model.state_dict()))
    model = model.to(dev)
    g = torch.Generator().manual_seed(0)
    x0 = (torch.rand(8, 3, 440, 1024, generator=g) * 2 - 1).to(dev)
    x1 = (torch.rand(8, 3, 440, 1024, generator=g) * 2 - 1).to(dev)
    arms = json.loads(os.environ.get("ARMS", '{"default": {}}'))
    from optical_flow import _native as N
    lib = N.load()
    hooks = sorted({h for v in arms.values() for h in v})
    out = {k: {"fnet_ms": [], "cnet_ms": [], "three_streams_ms": []} for k in arms}
    with torch.inference_mode():
        fnet, cnet = SplitEncoder(model.fnet), SplitEncoder(model.cnet)
        main_s = torch.cuda.current_stream(dev)
        s1, s2 = torch.cuda.Stream(dev), torch.cuda.Stream(dev)

        def three():
            s1.wait_stream(main_s)
            s2.wait_stream(main_s)
            with torch.cuda.stream(s1):
                fnet(x1, split_out=True, stem_from_image=True)
            with torch.cuda.stream(s2):
                cnet(x0, stem_from_image=True)
            fnet(x0, split_out=True, stem_from_image=True)
            main_s.wait_stream(s1)
            main_s.wait_stream(s2)
        for _ in range(int(os.environ.get("SAMPLES", "3"))):
            for k, v in arms.items():
                for h in hooks:
                    getattr(lib, h)(int(v.get(h, 0)))
                out[k]["fnet_ms"].append(timed(lambda: fnet(x0, split_out=True, stem_from_image=True), 10))
                out[k]["cnet_ms"].append(timed(lambda: cnet(x0, stem_from_image=True), 10))
                out[k]["three_streams_ms"].append(timed(three, 10))
        for h in hooks:
            getattr(lib, h)(0)
    out = {k: {m: round(statistics.median(t), 3) for m, t in v.items()} for k, v in out.items()}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
