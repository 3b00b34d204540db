"""Per-launch timing of one split encoder forward alone on the GPU (fnet: 8 Sintel images 440x1024, instance norm, S32
output; cnet: 8 images, folded batch norm): every oflow kernel launch of the forward is bracketed by events on its own
(the stream is synchronised between launches, so nothing overlaps), with its shapes and, for convolutions, executed
split-fp16 TFLOP/s (3 f16 MFMA products per MAC). Prints one JSON line per encoder."""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
for p in (REPO, os.path.join(REPO, "torch-optical-flow_amd"), os.path.join(REPO, "torch-optical-flow_amd", "methods", "raft")):
    sys.path.insert(0, p)

import torch  # noqa: E402

from optical_flow import _native as N  # noqa: E402
from model import RAFT, synthetic  # noqa: E402
from model.extractor import SplitEncoder  # noqa: E402

LOG = []


def wrap(name, fn, flops_fn=None):
    def inner(*args, **kw):
        torch.cuda.synchronize()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        r = fn(*args, **kw)
        b.record()
        torch.cuda.synchronize()
        us = a.elapsed_time(b) * 1e3
        ent = {"op": name, "us": round(us, 1)}
        if flops_fn is not None:
            ent.update(flops_fn(*args, **kw))
            if "gflop" in ent:
                ent["tflops"] = round(ent["gflop"] / us * 1e3 / 1e3, 1)
        LOG.append(ent)
        return r
    return inner


def conv_info(x, cw, block_n, *a, **kw):
    b, h, w = x.bhw
    mac = b * h * w * cw.n * cw.kg * 32 * cw.kh * cw.kw
    return {"in": type(x).__name__, "bhw": [b, h, w], "kg": cw.kg, "k": f"{cw.kh}x{cw.kw}", "n": cw.n, "bn": block_n,
            "stats": kw.get("stats") is not None, "gflop": round(6 * mac / 1e9, 2)}


def main():
    dev = torch.device("cuda", 0)
    model = RAFT().eval()
    model.load_state_dict(synthetic.synthetic_state_dict(model.state_dict()))
    model = model.to(dev)
    img0, _ = synthetic.synthetic_pair(8, 440, 1024, seed=0)
    x = (2 * (img0.to(dev) / 255.0) - 1.0).contiguous()
    N.conv_s32 = wrap("conv", N.conv_s32, conv_info)
    for nm in ("norm_apply", "norm_stats", "stem_patches", "pack_s32"):
        setattr(N, nm, wrap(nm, getattr(N, nm)))
    with torch.inference_mode():
        for name, enc, kw in (("fnet", model.fnet, {"split_out": True, "stem_from_image": True}),
                              ("cnet", model.cnet, {"stem_from_image": True})):
            se = SplitEncoder(enc)
            se(x, **kw)
            LOG.clear()
            se(x, **kw)
            tot = sum(e["us"] for e in LOG)
            print(json.dumps({"encoder": name, "total_us": round(tot, 1), "launches": list(LOG)}), flush=True)


if __name__ == "__main__":
    main()
