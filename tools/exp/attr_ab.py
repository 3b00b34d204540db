"""In-process A/B of RAFT model attributes on the Sintel x8 step (12 iterations, test mode): ATTRS (JSON) maps an arm
name to {attribute: value}; the arms run interleaved (3 forwards per sample, SAMPLES samples each), and the flows of
every arm are compared with the first arm's (bit-identical or max |d|). An attribute "lib:<symbol>" calls that
experiment hook of the native library with the value instead, "bn:<layer>" sets model.update.CONV_BN[layer]. Prints one JSON line.
  ATTRS='{"patch": {"stem_from_image": false}, "image": {"stem_from_image": true}}' python tools/exp/attr_ab.py"""
import json
import os
import statistics
import sys

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
for p in (REPO, os.path.join(REPO, "torch-optical-flow_amd"), os.path.join(REPO, "torch-optical-flow_amd", "methods", "raft")):
    sys.path.insert(0, p)

import torch  # noqa: E402

from model import RAFT, InputPadder, synthetic  # noqa: E402


def main():
    arms = json.loads(os.environ["ATTRS"])
    dev = torch.device("cuda", 0)
    model = RAFT().eval()
    model.load_state_dict(synthetic.synthetic_state_dict(model.state_dict()))
    model = model.to(dev)
    pairs = int(os.environ.get("PAIRS", "8"))
    a0, a1 = synthetic.synthetic_pair(2, 436, 1024, seed=0)
    padder = InputPadder((436, 1024), mode="sintel")
    reps = -(-pairs // 2)
    p0, p1 = padder.pad(a0.to(dev).repeat(reps, 1, 1, 1)[:pairs], a1.to(dev).repeat(reps, 1, 1, 1)[:pairs])
    res = {k: [] for k in arms}
    outs = {}

    from optical_flow import _native as N

    def setarm(k):
        for attr, v in arms[k].items():
            if attr.startswith("lib:"):  # an experiment hook of the native library: lib:<symbol> = int argument
                getattr(N.load(), attr[4:])(int(v))
            elif attr.startswith("native:"):  # a module constant of optical_flow._native (e.g. a kernel threshold)
                setattr(N, attr[7:], v)
            elif attr.startswith("mod:"):  # mod:<module>.<name>, e.g. mod:model.extractor.FOLD_BLOCK0
                import importlib
                mname, _, name = attr[4:].rpartition(".")
                setattr(importlib.import_module(mname), name, v)
            elif attr.startswith("bn:"):  # an update-block conv's output-channel block (model.update.CONV_BN)
                from model import update as U
                U.CONV_BN[attr[3:]] = int(v)
            else:  # a model attribute, or a dotted path to a sub-module's attribute (update_block.split_streams)
                obj = model
                *path, name = attr.split(".")
                for part in path:
                    obj = getattr(obj, part)
                setattr(obj, name, v)

    with torch.inference_mode():
        for k in arms:
            setarm(k)
            outs[k] = model(p0, p1, iters=12, test_mode=True)[1].clone()
            model(p0, p1, iters=12, test_mode=True)
        torch.cuda.synchronize()
        for _ in range(int(os.environ.get("SAMPLES", "6"))):
            for k in arms:
                setarm(k)
                a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                a.record()
                for _ in range(3):
                    model(p0, p1, iters=12, test_mode=True)
                b.record()
                b.synchronize()
                res[k].append(a.elapsed_time(b) / 3)
    first = next(iter(arms))
    out = {"pairs": pairs}
    for k in arms:
        d = (outs[k] - outs[first]).abs().max().item()
        out[k] = {"ms_median": round(statistics.median(res[k]), 3), "ms_min": round(min(res[k]), 3),
                  "max_abs_diff_vs_" + first: d}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
