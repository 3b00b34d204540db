"""In-process A/B of the LDS-staged warp's channels per workgroup (oflow_exp_set_warp_cpw: 0 = all channels in one
workgroup, 1 = one workgroup per channel, ...) on the SURVEY warp workload (8, 3, 436, 1024), flow normalize(N(0, 8^2))
px i.i.d. plus a smooth and a zero flow; outputs compared bit for bit across the settings. HOOK / CPW select another
hook and its settings (HOOK=oflow_exp_set_warp_strip CPW=1,0: strip-walking vs per-tile kernel). Prints JSON lines."""
import ctypes
import json
import os
import statistics
import sys

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
for p in (REPO, os.path.join(REPO, "torch-optical-flow_amd"), os.path.join(REPO, "torch-optical-flow_amd", "methods", "raft")):
    sys.path.insert(0, p)

import torch  # noqa: E402

import optical_flow  # noqa: E402
from optical_flow import _native as N  # noqa: E402
from model import synthetic  # noqa: E402

DEV = torch.device("cuda", 0)


def main():
    lib = N.load()
    hook = getattr(lib, os.environ.get("HOOK", "oflow_exp_set_warp_cpw"))  # e.g. HOOK=oflow_exp_set_warp_strip CPW=1,0
    hook.argtypes = [ctypes.c_int]
    b, c, h, w = 8, 3, 436, 1024
    flows = {}
    flows["iid8"] = [optical_flow.normalize(torch.from_numpy(synthetic.hash_normal(5 + k, (b, 2, h, w), 8.0))).to(DEV) for k in range(2)]
    yy, xx = torch.meshgrid(torch.arange(h), torch.arange(w), indexing="ij")
    sm = torch.stack([10 * torch.sin(xx / 37.0), 8 * torch.cos(yy / 23.0)]).float().unsqueeze(0).repeat(b, 1, 1, 1)
    flows["smooth"] = [optical_flow.normalize(sm).to(DEV)] * 2
    flows["zero"] = [torch.zeros(b, 2, h, w, device=DEV)] * 2
    frames = [synthetic.synthetic_pair(b, h, w, seed=1 + k)[0].to(DEV) for k in range(2)]
    nbytes = (2 * c + 2) * 4 * b * h * w
    settings = [int(v) for v in os.environ.get("CPW", "0,1,2").split(",")]
    with torch.inference_mode():
        for name, fl in flows.items():
            res, outs = {}, {}
            for cpw in settings:
                hook(cpw)
                outs[cpw] = optical_flow.warp(frames[0], fl[0]).clone()
            for _ in range(3):
                for cpw in settings:
                    hook(cpw)
                    ts = []
                    for i in range(20):
                        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                        e0.record()
                        optical_flow.warp(frames[i % 2], fl[i % 2])
                        e1.record()
                        torch.cuda.synchronize()
                        ts.append(e0.elapsed_time(e1) * 1e3)
                    res.setdefault(cpw, []).append(statistics.median(ts))
            hook(settings[0])
            same = all(torch.equal(outs[settings[0]], outs[k]) for k in settings)
            print(json.dumps({"flow": name, "bit_identical": same,
                              **{f"cpw{k}_us": round(min(v), 2) for k, v in res.items()},
                              **{f"cpw{k}_frac": round(nbytes / (min(v) * 1e-6) / 8e12, 4) for k, v in res.items()}}), flush=True)


if __name__ == "__main__":
    main()
