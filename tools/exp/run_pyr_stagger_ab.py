"""In-process A/B of a start stagger of the split-fp16 pyramid's first workgroups (experiment hook
oflow_exp_set_pyramid_stagger(cycles, mode): mode 1 delays workgroups 256-511 of image 0 -- the second workgroup slot
of every CU if the first 256 land one per CU --, mode 2 the odd ones below 512) at Sintel x8 (8 x 55 x 128, C = 256):
the two workgroups of a CU otherwise start together and stay in step, MFMA phase beside MFMA phase and store phase
beside store phase. Interleaved samples of 10 launches; every arm bit-identical. Prints one JSON line."""
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

ARMS = [(0, 1), (18000, 1), (37000, 2)] + ([(0, 5)] if os.environ.get('EPI_ONLY') else [])


def main():
    dev = torch.device("cuda", 0)
    g = torch.Generator(device="cpu").manual_seed(0)
    f1 = torch.randn((8, 256, 55, 128), generator=g).to(dev)
    f2 = torch.randn((8, 256, 55, 128), generator=g).to(dev)
    s1, s2 = N.s32_from_f32(f1), N.s32_from_f32(f2)
    lib = N.load()
    lib.oflow_exp_set_pyramid_stagger.argtypes = [ctypes.c_int, ctypes.c_int]
    ref = None
    same = True
    for arm in ARMS:
        lib.oflow_exp_set_pyramid_stagger(*arm)
        out = [t.clone() for t in N.corr_pyramid_tiled_s32(s1, s2, 4).levels]
        if ref is None:
            ref = out
        elif arm[1] & 4:
            pass  # the epilogue-only ablation stores zeros
        else:
            same = same and all(torch.equal(a, b) for a, b in zip(ref, out))
    del ref
    ts = {arm: [] for arm in ARMS}
    for _ in range(int(os.environ.get("SAMPLES", "8"))):
        for arm in ARMS:
            lib.oflow_exp_set_pyramid_stagger(*arm)
            torch.cuda.synchronize()
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            for _ in range(10):
                N.corr_pyramid_tiled_s32(s1, s2, 4)
            b.record()
            b.synchronize()
            ts[arm].append(a.elapsed_time(b) / 10)
    lib.oflow_exp_set_pyramid_stagger(0, 1)
    print(json.dumps({"bit_identical": same, "ms": {f"{c}c_m{m}": [round(statistics.median(v), 4), round(min(v), 4)]
                                                    for (c, m), v in ts.items()}}), flush=True)


if __name__ == "__main__":
    main()
