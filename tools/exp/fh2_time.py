"""Isolated timing of the flow head output conv (oflow_flow_head2_s32) at the Sintel 1/8 grid, batch 1 / 4 / 8."""
import json
import os
import statistics
import sys

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(REPO, "torch-optical-flow_amd"))
import torch  # noqa: E402

from optical_flow import _native as N  # noqa: E402

dev = torch.device("cuda", 0)
out = {}
for b in (1, 4, 8):
    x = torch.randn(b, 256, 55, 128, device=dev)
    xs = N.s32_from_f32(x)
    wt = torch.randn(2, 256, 3, 3, device=dev) / 48
    bias = torch.randn(2, device=dev)
    coords = torch.zeros(b, 2, 55, 128, device=dev)
    ts = []
    for it in range(40):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        N.flow_head2(N.S32Slice(xs), wt, bias, coords)
        e1.record()
        torch.cuda.synchronize()
        if it >= 5:
            ts.append(e0.elapsed_time(e1) * 1e3)
    out[f"b{b}"] = round(statistics.median(ts), 2)
print(json.dumps({"flow_head2_us": out}))
