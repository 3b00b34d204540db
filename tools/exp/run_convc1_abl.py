"""Ablations of the fused lookup + convc1 kernel (csrc/corr_convc1.hip), built here from textual variants of the
product source (nothing in the product carries the hooks): full; no MFMAs; no gathers (loads replaced by their offset);
no bilinear taps (one LDS read per slot); gathers only (no MFMAs, no taps). Sintel 55x128 grid, 8 pairs, cold pyramids.

    python tools/exp/run_convc1_abl.py build   # on the build host: writes tools/exp/lib/libc1abl_<v>.so
    python tools/exp/run_convc1_abl.py run     # on the GPU box
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
SRC = os.path.join(REPO, "torch-optical-flow_amd", "csrc", "corr_convc1.hip")
LIB = os.path.join(REPO, "tools", "exp", "lib")

MFMA = "__builtin_amdgcn_mfma_f32_32x32x16_f16("
VARIANTS = {
    "full": [],
    "nomfma": [("acc[mt][nt] = " + MFMA, "acc[mt][nt] = nomfma(")],
    "nogather": [("__builtin_amdgcn_raw_buffer_load_b32(rs, off, 0, 0)", "(unsigned)off")],
    "notaps": [("v = bilinear4(p[j * PK + i], p[j * PK + i + 1], p[(j + 1) * PK + i], p[(j + 1) * PK + i + 1], w4);",
                "v = p[j * PK + i];")],
    "gatheronly": [("acc[mt][nt] = " + MFMA, "acc[mt][nt] = nomfma("),
                   ("v = bilinear4(p[j * PK + i], p[j * PK + i + 1], p[(j + 1) * PK + i], p[(j + 1) * PK + i + 1], w4);",
                    "v = p[j * PK + i];")],
    "noweights": [("rb[s] = *reinterpret_cast<const u32x4*>(wg + (size_t)(tid + kNT * s) * 16);",
                   "rb[s] = u32x4{(unsigned)s, (unsigned)g, 0u, 0u};")],
    "nobarrier": [("__syncthreads();  // group g's", "//"), ("__syncthreads();  // patches dead", "//")],
    "nostore": [("*reinterpret_cast<half8*>(line) = hi;", "if (hi[0] == (_Float16)12345.f) *reinterpret_cast<half8*>(line) = hi;"),
                ("*reinterpret_cast<half8*>(line + 64) = lo;", "")],
}
NOMFMA = """
__device__ __forceinline__ f32x16 nomfma(half8 a, half8 b, f32x16 c, int, int, int) {
  c[0] += (float)a[0] * (float)b[0];
  return c;
}
"""


def build():
    os.makedirs(LIB, exist_ok=True)
    src = open(SRC).read()
    for name, subs in VARIANTS.items():
        s = src
        for a, b in subs:
            assert a in s, (name, a)
            s = s.replace(a, b)
        s = s.replace("__device__ __forceinline__ int swz(int row)", NOMFMA + "__device__ __forceinline__ int swz(int row)")
        s = s.replace("oflow_corr_lookup_convc1_s32", f"abl_{name}")
        path = f"/tmp/c1abl_{name}.hip"
        open(path, "w").write(s)
        inc = os.path.join(REPO, "torch-optical-flow_amd", "csrc")
        subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared",
                        "-fno-slp-vectorize", "-fno-vectorize", f"-I{inc}", f"-I{os.path.join(REPO, 'include')}",
                        path, "-o", os.path.join(LIB, f"libc1abl_{name}.so")], check=True)
        print("built", name)


def run():
    import torch

    from optical_flow import _native as N
    from model import synthetic
    from model.utils import coords_grid

    dev = torch.device("cuda", 0)
    b, h, w = 8, 55, 128
    pyrs = []
    for k in range(3):
        f1, f2 = synthetic.synthetic_fmaps(b, 256, h, w, stream=k)
        pyrs.append(N.corr_pyramid_tiled(f1.to(dev), f2.to(dev), 4))
    coords = (coords_grid(b, h, w) + torch.from_numpy(synthetic.hash_normal(9, (b, 2, h, w), 4.0))).to(dev).contiguous()
    conv = torch.nn.Conv2d(324, 256, 1).to(dev)
    cw = N.convc1_level_weights(conv, 4, 4)
    y = N.s32_empty(b, h, w, 8, dev)
    P = ctypes.c_void_p
    out = {}
    for name in VARIANTS:
        lib = ctypes.CDLL(os.path.join(LIB, f"libc1abl_{name}.so"))
        fn = getattr(lib, f"abl_{name}")
        fn.restype = ctypes.c_int
        fn.argtypes = [P, P, P, ctypes.c_int, P, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, P, P, P, P,
                       ctypes.c_longlong, P]
        hs = (ctypes.c_int * 8)(*[d[0] for d in pyrs[0].dims])
        ws = (ctypes.c_int * 8)(*[d[1] for d in pyrs[0].dims])
        ptrs = [(ctypes.c_void_p * 8)(*[t.data_ptr() for t in pp.levels]) for pp in pyrs]
        st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
        ts = []
        for it in range(24):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            rc = fn(ptrs[it % 3], hs, ws, 4, coords.data_ptr(), b, h, w, 4, cw.pack.data_ptr(), cw.wscale.data_ptr(),
                    cw.bias.data_ptr(), y.ptr if hasattr(y, "ptr") else y.data_ptr(), 1024, st)
            e1.record()
            torch.cuda.synchronize()
            assert rc == 0, rc
            if it >= 4:
                ts.append(e0.elapsed_time(e1) * 1e3)
        out[name] = round(statistics.median(ts), 2)
        if name == "full":  # per-level cost: the same kernel over 1 and 2 levels, and over one 256-workgroup round
            for nl in (1, 2):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                tt = []
                for it in range(12):
                    e0.record()
                    fn(ptrs[it % 3], hs, ws, nl, coords.data_ptr(), b, h, w, 4, cw.pack.data_ptr(), cw.wscale.data_ptr(),
                       cw.bias.data_ptr(), y.ptr if hasattr(y, "ptr") else y.data_ptr(), 1024, st)
                    e1.record()
                    torch.cuda.synchronize()
                    tt.append(e0.elapsed_time(e1) * 1e3)
                out[f"full_levels{nl}"] = round(statistics.median(tt[2:]), 2)
            tt = []
            for it in range(12):  # 2 rows of 128 px per workgroup... one image of 55x128 x 4 pairs = 220 workgroups
                e0.record()
                fn(ptrs[it % 3], hs, ws, 4, coords.data_ptr(), 4, h, w, 4, cw.pack.data_ptr(), cw.wscale.data_ptr(),
                   cw.bias.data_ptr(), y.ptr if hasattr(y, "ptr") else y.data_ptr(), 1024, st)
                e1.record()
                torch.cuda.synchronize()
                tt.append(e0.elapsed_time(e1) * 1e3)
            out["full_4pairs_220wg"] = round(statistics.median(tt[2:]), 2)
    print(json.dumps({"convc1_ablation_us_sintel8": out}))


if __name__ == "__main__":
    {"build": build, "run": run}[sys.argv[1]]()
