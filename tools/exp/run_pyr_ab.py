"""In-process A/B of the split-fp16 pyramid's level-0/1 store policy (plain vs non-temporal, experiment hook
oflow_exp_set_pyramid_nt) at Sintel x8 (8 x 55 x 128, C = 256): interleaved samples of 10 launches each; the levels of
both arms must be bit-identical. Prints one JSON line."""
import ctypes
import json
import os
import statistics
import sys

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
for p in (REPO, os.path.join(REPO, "torch-optical-flow_amd")):
    sys.path.insert(0, p)

import torch  # noqa: E402

from optical_flow import _native as N  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    g = torch.Generator(device="cpu").manual_seed(0)
    f1 = torch.randn((8, 256, 55, 128), generator=g).to(dev)
    f2 = torch.randn((8, 256, 55, 128), generator=g).to(dev)
    s1, s2 = N.s32_from_f32(f1), N.s32_from_f32(f2)
    lib = N.load()
    lib.oflow_exp_set_pyramid_nt.argtypes = [ctypes.c_int]
    outs, ts = {}, {0: [], 1: []}
    for arm in (0, 1):
        lib.oflow_exp_set_pyramid_nt(arm)
        outs[arm] = [t.clone() for t in N.corr_pyramid_tiled_s32(s1, s2, 4).levels]
    same = all(torch.equal(a, b) for a, b in zip(outs[0], outs[1]))
    del outs
    for _ in range(int(os.environ.get("SAMPLES", "8"))):
        for arm in (0, 1):
            lib.oflow_exp_set_pyramid_nt(arm)
            torch.cuda.synchronize()
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            for _ in range(10):
                N.corr_pyramid_tiled_s32(s1, s2, 4)
            b.record()
            b.synchronize()
            ts[arm].append(a.elapsed_time(b) / 10)
    lib.oflow_exp_set_pyramid_nt(0)
    print(json.dumps({"bit_identical": same, "plain_ms": round(statistics.median(ts[0]), 4),
                      "nt_ms": round(statistics.median(ts[1]), 4), "plain_min": round(min(ts[0]), 4),
                      "nt_min": round(min(ts[1]), 4)}), flush=True)


if __name__ == "__main__":
    main()
