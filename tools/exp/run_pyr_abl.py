"""Ablations of the split-fp16 pyramid kernel (csrc/corr_pyramid.hip, corr_pyramid_s32_kernel), built from textual
variants of the product source: full; no epilogue stores; no MFMAs; no global loads in the main loop. Sintel x8.

    python tools/exp/run_pyr_abl.py build   # build host: tools/exp/lib/libpyrabl_<v>.so
    python tools/exp/run_pyr_abl.py run     # GPU box
"""
import ctypes
import json
import os
import statistics
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
for p in (REPO, os.path.join(REPO, "torch-optical-flow_amd"), os.path.join(REPO, "torch-optical-flow_amd", "methods", "raft")):
    sys.path.insert(0, p)
SRC = os.path.join(REPO, "torch-optical-flow_amd", "csrc", "corr_pyramid.hip")
LIB = os.path.join(REPO, "tools", "exp", "lib")
MF = "acc[n] = __builtin_amdgcn_mfma_f32_32x32x16_f16("
VARIANTS = {
    "full": [],
    "noepi": [("  pyramid_epilogue<TILED>(p, acc, i0, ty0, tx0, b, reinterpret_cast<float*>(sB));\n}\n\n// Levels",
               "  if (acc[0][0] == 12345.f) p.lv[0][threadIdx.x] = acc[1][1];\n}\n\n// Levels")],
    "nomfma": [(MF + "ah, bl", "acc[n] = nomf(ah, bl"), (MF + "al, bh", "acc[n] = nomf(al, bh"), (MF + "ah, bh", "acc[n] = nomf(ah, bh")],
    "noload": [("ra[s] = *reinterpret_cast<const u32x4*>(A0 + aoff[s] + g * 128);", "ra[s] = u32x4{(unsigned)g, 1u, 2u, 3u};"),
               ("rb[s] = *reinterpret_cast<const u32x4*>(B0 + boff[s] + g * 128);", "rb[s] = u32x4{(unsigned)g, 3u, 2u, 1u};")],
}
NOMF = """
typedef _Float16 abl_half8 __attribute__((ext_vector_type(8)));
__device__ __forceinline__ f32x16 nomf(abl_half8 a, abl_half8 b, f32x16 c, int, int, int) { c[0] += (float)a[0] * (float)b[0]; return c; }
"""


def build():
    os.makedirs(LIB, exist_ok=True)
    src = open(SRC).read()
    for name, subs in VARIANTS.items():
        s = src
        for a, b in subs:
            assert a in s, (name, a)
            s = s.replace(a, b)
        s = s.replace("// Workgroup -> (target tile, query block)", NOMF + "// Workgroup -> (target tile, query block)")
        s = s.replace("oflow_corr_pyramid_tiled_s32", f"abl_{name}")
        for sym in ("oflow_corr_tiled_level_floats", "oflow_corr_untile_f32", "oflow_corr_pyramid_dims", "oflow_corr_pyramid_f32",
                    "oflow_corr_pyramid_tiled_f32"):
            s = s.replace(sym, f"{sym}_abl_{name}")
        s = s.replace("oflow_corr_pyramid_dims_abl_" + name + "(H, W, num_levels, hl, wl)", "oflow_corr_pyramid_dims_abl_" + name + "(H, W, num_levels, hl, wl)")
        path = f"/tmp/pyrabl_{name}.hip"
        open(path, "w").write(s)
        inc = os.path.join(REPO, "torch-optical-flow_amd", "csrc")
        subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared",
                        "-fno-slp-vectorize", "-fno-vectorize", f"-I{inc}", f"-I{os.path.join(REPO, 'include')}",
                        path, "-o", os.path.join(LIB, f"libpyrabl_{name}.so")], check=True)
        print("built", name)


def run():
    import torch

    from optical_flow import _native as N
    from model import synthetic

    dev = torch.device("cuda", 0)
    b, h, w = 8, 55, 128
    f1, f2 = synthetic.synthetic_fmaps(b, 256, h, w, stream=3)
    s1, s2 = N.s32_from_f32(f1.to(dev)), N.s32_from_f32(f2.to(dev))
    pyr = N.corr_pyramid_tiled_s32(s1, s2, 4)
    ptrs = (ctypes.c_void_p * 8)(*[t.data_ptr() for t in pyr.levels])
    P, I = ctypes.c_void_p, ctypes.c_int
    out = {}
    for name in VARIANTS:
        lib = ctypes.CDLL(os.path.join(LIB, f"libpyrabl_{name}.so"))
        fn = getattr(lib, f"abl_{name}")
        fn.restype = I
        fn.argtypes = [P, P, I, I, I, I, I, ctypes.POINTER(ctypes.c_void_p), P]
        st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
        ts = []
        for it in range(14):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            rc = fn(s1.data_ptr(), s2.data_ptr(), b, 256, h, w, 4, ptrs, st)
            e1.record()
            torch.cuda.synchronize()
            assert rc == 0, rc
            if it >= 4:
                ts.append(e0.elapsed_time(e1) * 1e3)
        out[name] = round(statistics.median(ts), 1)
    print(json.dumps({"pyramid_s32_ablation_us_sintel8": out}))


if __name__ == "__main__":
    {"build": build, "run": run}[sys.argv[1]]()
