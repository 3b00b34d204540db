"""In-process A/B of one split encoder (fnet: instance norm, S32 output; cnet: batch norm) on 8 Sintel images
(440x1024): the stem from a patch matrix vs from the image (stem_from_image). Interleaved, median of 10 per round x 3,
outputs compared bit for bit. Prints one JSON line."""
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


def main():
    dev = torch.device("cuda", 0)
    model = RAFT().eval()
    model.load_state_dict(synthetic.synthetic_state_dict(model.state_dict()))
    model = model.to(dev)
    img0, _ = synthetic.synthetic_pair(8, 440, 1024, seed=0)
    x = (2 * (img0.to(dev) / 255.0) - 1.0).contiguous()
    out = {}
    with torch.inference_mode():
        for name, enc, kw in (("fnet", model.fnet, {"split_out": True}), ("cnet", model.cnet, {})):
            se = SplitEncoder(enc)
            arms = {"patch": dict(kw), "image": dict(kw, stem_from_image=True)}
            res = {k: se(x, **a).clone() for k, a in arms.items()}
            ts = {k: [] for k in arms}
            for _ in range(3):
                for k, a in arms.items():
                    e = []
                    for _ in range(10):
                        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                        e0.record()
                        se(x, **a)
                        e1.record()
                        torch.cuda.synchronize()
                        e.append(e0.elapsed_time(e1))
                    ts[k].append(statistics.median(e))
            out[name] = {"bit_identical": torch.equal(res["patch"], res["image"]),
                         **{f"{k}_ms": round(min(v), 3) for k, v in ts.items()}}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
