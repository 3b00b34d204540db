"""A/B of the split pyramid's target-tile order (Sintel x8, C = 256): blocked 4x2 target tiles (default) vs row-major
(oflow_exp_set_pyramid_stagger mode bit 7), full kernel and epilogue alone (bit 2), interleaved samples; levels
compared bit for bit between the orders; plus the fp32 API pyramid (CorrBlock) at configs[1]. One JSON line.
The blocked order (mode bit 7) was removed after this run (profiles/r05/s41_pyr_order.log)."""
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
    f1, f2 = torch.randn((8, 256, 55, 128), generator=g).to(dev), torch.randn((8, 256, 55, 128), generator=g).to(dev)
    s1, s2 = N.s32_from_f32(f1), N.s32_from_f32(f2)
    lib = N.load()
    lib.oflow_exp_set_pyramid_stagger.argtypes = [ctypes.c_int, ctypes.c_int]
    levels = {}
    for mode in (1, 129):
        lib.oflow_exp_set_pyramid_stagger(0, mode)
        levels[mode] = [t.clone() for t in N.corr_pyramid_tiled_s32(s1, s2, 4).levels]
    same = all(torch.equal(a, b) for a, b in zip(levels[1], levels[129]))
    del levels
    arms = {"blocked": 1, "rowmajor": 129, "blocked_epi": 5, "rowmajor_epi": 133}
    ts = {k: [] for k in arms}
    for _ in range(8):
        for name, mode in arms.items():
            lib.oflow_exp_set_pyramid_stagger(0, mode)
            torch.cuda.synchronize()
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            for _ in range(10):
                N.corr_pyramid_tiled_s32(s1, s2, 4)
            b.record()
            b.synchronize()
            ts[name].append(a.elapsed_time(b) / 10)
    out = {"bit_identical": same, "ms": {k: [round(statistics.median(v), 4), round(min(v), 4)] for k, v in ts.items()}}
    # the fp32 API pyramid at configs[1] (4 x 256 x 128 x 128)
    a1, a2 = torch.randn((4, 256, 128, 128), generator=g).to(dev), torch.randn((4, 256, 128, 128), generator=g).to(dev)
    fp = {}
    for name, mode in (("blocked", 1), ("rowmajor", 129)):
        lib.oflow_exp_set_pyramid_stagger(0, mode)
        N.corr_pyramid_tiled(a1, a2, 4)
        torch.cuda.synchronize()
        v = []
        for _ in range(5):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            for _ in range(5):
                N.corr_pyramid_tiled(a1, a2, 4)
            b.record()
            b.synchronize()
            v.append(a.elapsed_time(b) / 5)
        fp[name] = round(statistics.median(v), 4)
    lib.oflow_exp_set_pyramid_stagger(0, 1)
    out["fp32_configs1_ms"] = fp
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
