"""The bench's two after-the-step legs alone, for A/B of library builds in separate processes (OFLOW_LIB=...): the API
lookup (CorrBlock.__call__ at the Sintel x8 shapes, coordinates = grid + the synthetic frames' (3, -1.5) px shift at
1/8 resolution + N(0, 0.5^2)) and the warp (8, 3, 436, 1024), each as bench.py times it (launches queued behind a spin
kernel). Prints one JSON line; REPS rounds, medians."""
import json
import os
import statistics
import sys

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
for p in (REPO, os.path.join(REPO, "torch-optical-flow_amd"), os.path.join(REPO, "torch-optical-flow_amd", "methods", "raft")):
    sys.path.insert(0, p)

import torch  # noqa: E402

import bench  # noqa: E402
from model import synthetic  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    b, h, w = 8, 55, 128
    dims = [(h >> l, w >> l) for l in range(4)]
    flow = torch.from_numpy(synthetic.hash_normal(11, (b, 2, h, w), 0.5))
    flow[:, 0] += 3.0 / 8
    flow[:, 1] -= 1.5 / 8
    flow = flow.to(dev)
    lk, wp = [], []
    for _ in range(int(os.environ.get("REPS", "5"))):
        lk.append(bench.lookup_api_leg(b, dims, flow, dev)["launch_ms"])
        wp.append(bench.warp_leg(dev)["launch_ms"])
    lms, wms = statistics.median(lk), statistics.median(wp)
    nb = bench.lookup_bytes(b, dims)
    print(json.dumps({"lib": os.environ.get("OFLOW_LIB", "in-tree"), "lookup_us": round(lms * 1e3, 2),
                      "lookup_frac": round(nb / (lms * 1e-3) / 8e12, 4), "warp_us": round(wms * 1e3, 2),
                      "warp_frac": round((2 * 3 + 2) * 4 * 8 * 436 * 1024 / (wms * 1e-3) / 8e12, 4)}), flush=True)


if __name__ == "__main__":
    main()
