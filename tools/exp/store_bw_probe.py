"""HBM store-bandwidth reference for the split pyramid's epilogue: a 2.11 GB fill (torch fill_: plain wide stores), a
2.11 GB copy, and the pyramid (Sintel x8, C = 256) in full and with its main loop removed (oflow_exp_set_pyramid_stagger
mode bit 2: the epilogue alone, storing the same 2.11 GB of levels). Median of 8 samples of 10 launches. One JSON line."""
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


def timed(fn, samples=8, reps=10):
    ts = []
    for _ in range(samples):
        torch.cuda.synchronize()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(reps):
            fn()
        b.record()
        b.synchronize()
        ts.append(a.elapsed_time(b) / reps)
    return statistics.median(ts)


def main():
    dev = torch.device("cuda", 0)
    g = torch.Generator(device="cpu").manual_seed(0)
    f1 = torch.randn((8, 256, 55, 128), generator=g).to(dev)
    f2 = torch.randn((8, 256, 55, 128), generator=g).to(dev)
    s1, s2 = N.s32_from_f32(f1), N.s32_from_f32(f2)
    lib = N.load()
    lib.oflow_exp_set_pyramid_stagger.argtypes = [ctypes.c_int, ctypes.c_int]
    pyr = N.corr_pyramid_tiled_s32(s1, s2, 4)
    nbytes = sum(t.numel() * 4 for t in pyr.levels)
    del pyr
    buf = torch.empty(nbytes // 4, device=dev, dtype=torch.float32)
    src = torch.empty_like(buf).fill_(1.0)
    out = {"bytes": nbytes}
    ms = timed(lambda: buf.fill_(0.5))
    out["fill"] = {"ms": round(ms, 4), "TB/s": round(nbytes / ms / 1e9, 2)}
    ms = timed(lambda: buf.copy_(src))
    out["copy"] = {"ms": round(ms, 4), "TB/s (read+write)": round(2 * nbytes / ms / 1e9, 2)}
    del src, buf
    for name, mode in (("pyramid", 1), ("pyramid_epilogue_only", 5)):
        lib.oflow_exp_set_pyramid_stagger(0, mode)
        ms = timed(lambda: N.corr_pyramid_tiled_s32(s1, s2, 4))
        out[name] = {"ms": round(ms, 4), "TB/s of stores": round(nbytes / ms / 1e9, 2)}
    lib.oflow_exp_set_pyramid_stagger(0, 1)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
