"""Per-kernel timing events inside a captured HIP graph with liboflow's native timing events (N.TimingEvent: external
event-record nodes; torch.cuda.Event(external=True) is refused on ROCm, tools/exp/graph_event_probe.py): captures
[event a] fused lookup + convc1 [event b] x 3, replays, and compares a.elapsed_time(b) with eager timing of the same
launch. Prints one JSON line."""
import json
import os
import statistics
import sys

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
for p in (REPO, os.path.join(REPO, "torch-optical-flow_amd"), os.path.join(REPO, "torch-optical-flow_amd", "methods", "raft")):
    sys.path.insert(0, p)

import torch  # noqa: E402

from optical_flow import _native as N  # noqa: E402
from model import synthetic  # noqa: E402
from model.utils import coords_grid  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    b, h, w = 4, 55, 128
    conv = torch.nn.Conv2d(324, 256, 1).to(dev)
    cw = N.convc1_level_weights(conv, 4, 4)
    f1, f2 = synthetic.synthetic_fmaps(b, 256, h, w, stream=0)
    pyr = N.corr_pyramid_tiled(f1.to(dev), f2.to(dev), 4)
    coords = (coords_grid(b, h, w) + torch.from_numpy(synthetic.hash_normal(9, (b, 2, h, w), 4.0))).to(dev).contiguous()
    y = N.s32_empty(b, h, w, 8, dev)
    out = {}
    with torch.inference_mode():
        eager = []
        for _ in range(10):
            a, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            N.corr_lookup_convc1(pyr, coords, 4, cw, N.S32Slice(y))
            e.record()
            e.synchronize()
            eager.append(a.elapsed_time(e) * 1e3)
        out["eager_us"] = round(statistics.median(eager), 2)
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            N.corr_lookup_convc1(pyr, coords, 4, cw, N.S32Slice(y))
        torch.cuda.synchronize()
        evs = [(N.TimingEvent(), N.TimingEvent()) for _ in range(3)]
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=s):
            for a, e in evs:
                a.record(s)
                N.corr_lookup_convc1(pyr, coords, 4, cw, N.S32Slice(y))
                e.record(s)
        print("captured", flush=True)
        reps = []
        for _ in range(5):
            g.replay()
            torch.cuda.synchronize()
            reps.append([round(a.elapsed_time(e) * 1e3, 2) for a, e in evs])
        out["graph_us"] = reps
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
