"""Ablations of the split pyramid's epilogue (Sintel x8, C = 256; oflow_exp_set_pyramid_stagger mode bits: 4 = no main
loop, 8 = level 0 alone, 16 = level 0 stored straight from the accumulators, unstaged, 32 / 64 = no level-3 / level 1-3
stores) against a 2.11 GB fill, to find
what holds its stores at ~3.8 TB/s. Median of 8 samples of 10 launches. One JSON line."""
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
from store_bw_probe import timed  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    g = torch.Generator(device="cpu").manual_seed(0)
    s1 = N.s32_from_f32(torch.randn((8, 256, 55, 128), generator=g).to(dev))
    s2 = N.s32_from_f32(torch.randn((8, 256, 55, 128), generator=g).to(dev))
    lib = N.load()
    lib.oflow_exp_set_pyramid_stagger.argtypes = [ctypes.c_int, ctypes.c_int]
    pyr = N.corr_pyramid_tiled_s32(s1, s2, 4)
    lv_bytes = [t.numel() * 4 for t in pyr.levels]
    del pyr
    out = {"level_bytes": lv_bytes}
    arms = {"full": 1, "epi": 5, "epi_l0": 13, "epi_no_l3_stores": 37, "epi_no_l123_stores": 69, "full_no_l3_stores": 33,
            "full_no_l123_stores": 65}
    for name, mode in arms.items():
        lib.oflow_exp_set_pyramid_stagger(0, mode)
        ms = timed(lambda: N.corr_pyramid_tiled_s32(s1, s2, 4))
        nb = lv_bytes[0] if mode & 72 else sum(lv_bytes[:3]) if mode & 32 else sum(lv_bytes)
        out[name] = {"ms": round(ms, 4), "TB/s": round(nb / ms / 1e9, 2)}
    lib.oflow_exp_set_pyramid_stagger(0, 1)
    buf = torch.empty(lv_bytes[0] // 4, device=dev)
    ms = timed(lambda: buf.fill_(0.5))
    out["fill_l0_bytes"] = {"ms": round(ms, 4), "TB/s": round(lv_bytes[0] / ms / 1e9, 2)}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
