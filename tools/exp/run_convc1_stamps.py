"""The fused lookup + convc1 kernel (oflow_corr_lookup_convc1_s32) alone on the Sintel 55x128 grid, 4 pairs (one pair
lane's launch) and 8 pairs, N(0, 4^2) px flow, three pyramids in rotation (cold in the 256 MiB Infinity Cache): median
of 20 event-timed launches x 3 rounds, then one launch with per-workgroup clock stamps (oflow_exp_set_convc1_stamps;
s_memtime is per XCD, so only in-workgroup differences are used): median cycles per phase. Run with OFLOW_LIB /
OFLOW_OPS_LIB pointing at another build (tools/build_rev.sh) for a back-to-back A/B. Prints JSON lines."""
import ctypes
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

DEV = torch.device("cuda", 0)


def timeit(fn, reps=20):
    ts = []
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        torch.cuda.synchronize()
        ts.append(a.elapsed_time(b) * 1e3)
    return statistics.median(ts)


def main():
    lib = N.load()
    stamps_hook = getattr(lib, "oflow_exp_set_convc1_stamps", None)
    if stamps_hook is not None:
        stamps_hook.argtypes = [ctypes.c_void_p]
    h, w = 55, 128
    conv = torch.nn.Conv2d(324, 256, 1).to(DEV)
    cwL = N.convc1_level_weights(conv, 4, 4)
    out = {"lib": N.library_path()}
    with torch.inference_mode():
        for b in (4, 8):
            pyrs = []
            for k in range(3):
                f1, f2 = synthetic.synthetic_fmaps(b, 256, h, w, stream=k)
                pyrs.append(N.corr_pyramid_tiled(f1.to(DEV), f2.to(DEV), 4))
            coords = (coords_grid(b, h, w) + torch.from_numpy(synthetic.hash_normal(9, (b, 2, h, w), 4.0))).to(DEV).contiguous()
            y = N.s32_empty(b, h, w, 8, DEV)
            it = [0]

            def fused():
                it[0] = (it[0] + 1) % 3
                N.corr_lookup_convc1(pyrs[it[0]], coords, 4, cwL, N.S32Slice(y))

            for _ in range(3):
                fused()
            torch.cuda.synchronize()
            out[f"pairs{b}_us"] = round(min(timeit(fused) for _ in range(3)), 2)
            if stamps_hook is not None:
                nwg = (b * h * w + 63) // 64
                st = torch.zeros(nwg * 16, dtype=torch.int64, device=DEV)
                stamps_hook(st.data_ptr())
                fused()
                torch.cuda.synchronize()
                stamps_hook(None)
                t = st.view(nwg, 16).cpu().double()
                names = ["prologue"] + [f"L{l}{ph}" for l in range(4) for ph in ("wait+patch", "gather+taps", "mfma")] + ["epilogue"]
                ph = {nm: round(float((t[:, i + 1] - t[:, i]).median())) for i, nm in enumerate(names)}
                ph["wg_life"] = round(float((t[:, 14] - t[:, 0]).median()))
                out[f"pairs{b}_stamps_cycles"] = ph
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
