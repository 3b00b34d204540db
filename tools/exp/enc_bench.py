"""Time the split encoders alone (Sintel x8 padded to 440x1024): fnet on one image batch, cnet on one, and the three
encoder streams of the RAFT forward (fnet image0 | fnet image1 | cnet image0) together. Prints one JSON line.
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
    out = {}
    with torch.inference_mode():
        fnet, cnet = SplitEncoder(model.fnet), SplitEncoder(model.cnet)
        out["fnet_ms"] = timed(lambda: fnet(x0, split_out=True, stem_from_image=True))
        out["cnet_ms"] = timed(lambda: cnet(x0, stem_from_image=True))
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
        out["three_streams_ms"] = timed(three)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
