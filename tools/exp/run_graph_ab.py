"""In-process A/B of update-block settings on the benchmarked forward (8 Sintel pairs, two lanes, 12 iterations, replayed
from a HIP graph as bench.py --graph does): one GraphedRAFT per variant, each captured with its module attributes set,
then replays alternated variant by variant for ROUNDS rounds (median ms per step per variant). Flows are compared with
the first variant's.

    VARIANTS='off:update.KSPLIT_LAYERS=frozenset();on:update.KSPLIT_LAYERS=frozenset({"mo","q"})' \
        python tools/exp/run_graph_ab.py
Each variant is "name:module.ATTR=python-expression[,,module.ATTR=...]" over the modules of methods/raft/model, or
"lib.oflow_exp_set_X=V/R": liboflow's int experiment setter, V during the capture, R after it."""
import ctypes
import importlib
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
from optical_flow import _native  # noqa: E402


class _Lib:
    """lib.oflow_exp_set_X=V/R: the library's int setter, called with V for the capture and R after it."""

    def __init__(self):
        self.vals = {}

    def set(self, name, v):
        fn = getattr(_native.load(), name)
        fn.argtypes, fn.restype = [ctypes.c_int], None
        fn(int(v))
        self.vals[name] = v


def parse(spec):
    out = []
    for item in filter(None, spec.split(";")):
        name, _, sets = item.partition(":")
        assigns = []
        for a in filter(None, sets.split(",,")):
            lhs, _, rhs = a.partition("=")
            mod, _, attr = lhs.strip().rpartition(".")
            if mod == "lib":
                v, _, r = rhs.partition("/")
                assigns.append(("lib", attr, (int(v), int(r or 0))))
            else:
                assigns.append((importlib.import_module("model." + mod), attr, eval(rhs)))  # noqa: S307 (experiment tool)
        out.append((name, assigns))
    return out


def main():
    variants = parse(os.environ.get("VARIANTS", ""))
    rounds = int(os.environ.get("ROUNDS", "6"))
    reps = int(os.environ.get("REPS", "20"))
    pairs = int(os.environ.get("PAIRS", "8"))
    dev = torch.device("cuda", 0)
    model = RAFT().eval()
    model.load_state_dict(synthetic.synthetic_state_dict(model.state_dict()))
    model = model.to(dev)
    a0, a1 = synthetic.synthetic_pair(2, 436, 1024, seed=0)
    padder = InputPadder((436, 1024), mode="sintel")
    r = -(-pairs // 2)
    p0, p1 = padder.pad(a0.to(dev).repeat(r, 1, 1, 1)[:pairs], a1.to(dev).repeat(r, 1, 1, 1)[:pairs])
    graphs, flows = {}, {}
    with torch.inference_mode():
        lib = _Lib()
        for name, assigns in variants:
            saved = [(m, at, getattr(m, at)) for m, at, _ in assigns if m != "lib"]
            for m, at, v in assigns:
                if m == "lib":
                    lib.set(at, v[0])
                else:
                    setattr(m, at, v)
            try:
                graphs[name] = G.GraphedRAFT(model, p0, p1, iters=12)
                flows[name] = graphs[name](p0, p1)[1].clone()
            finally:
                for m, at, v in saved:
                    setattr(m, at, v)
                for m, at, v in assigns:
                    if m == "lib":
                        lib.set(at, v[1])
        torch.cuda.synchronize()
        times = {n: [] for n in graphs}
        for _ in range(rounds):
            for n, g in graphs.items():
                g(p0, p1)
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(reps):
                    g(p0, p1)
                e1.record()
                e1.synchronize()
                times[n].append(e0.elapsed_time(e1) / reps)
    first = next(iter(flows))
    out = {"pairs": pairs, "rounds": rounds, "reps": reps}
    for n in graphs:
        ms = statistics.median(times[n])
        epe = torch.norm(flows[n] - flows[first], dim=1)
        out[n] = {"ms_per_step": round(ms, 3), "pairs_per_s": round(pairs * 1000 / ms, 1),
                  "min_ms": round(min(times[n]), 3), "epe_vs_first_mean": float(epe.mean()), "epe_vs_first_max": float(epe.max()),
                  "bit_identical_to_first": bool(torch.equal(flows[n], flows[first]))}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
