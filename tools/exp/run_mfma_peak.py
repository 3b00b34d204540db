"""EXPERIMENT: sustained f16 MFMA rate (32x32x16, 3 dependent MFMAs per accumulator as in conv_s32) on the whole chip."""
import ctypes
import json
import os

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
lib = ctypes.CDLL(os.path.join(HERE, "libmfma_peak.so"))
VP = ctypes.c_void_p


def main():
    dev = torch.device("cuda", 0)
    src = (torch.rand(1024 * 8, device=dev) * 2 - 1).half()
    res = {}
    for nacc in (4, 8):
        for blocks in (256, 512, 1024):  # 1, 2, 4 waves per SIMD (4 waves per block, 256 CUs)
            out = torch.empty(blocks * 256, device=dev)
            iters = 2000
            st = VP(torch.cuda.current_stream().cuda_stream)
            lib.exp_mfma(nacc, VP(src.data_ptr()), VP(out.data_ptr()), blocks, 10, st)
            torch.cuda.synchronize()
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            lib.exp_mfma(nacc, VP(src.data_ptr()), VP(out.data_ptr()), blocks, iters, st)
            b.record()
            b.synchronize()
            ms = a.elapsed_time(b)
            mfmas = blocks * 4 * iters * nacc * 3
            flops = mfmas * 32 * 32 * 16 * 2
            res[f"nacc{nacc}_blocks{blocks}"] = {"ms": round(ms, 3), "TFLOPs": round(flops / ms / 1e9, 1),
                                                  "cycles_per_mfma_at_2.4GHz": round(ms * 1e-3 * 2.4e9 * 1024 / mfmas, 1)}
            print(f"nacc{nacc} blocks{blocks}", res[f"nacc{nacc}_blocks{blocks}"], flush=True)
    srcf = torch.rand(1024 * 8, device=dev) * 2 - 1
    for blocks in (256, 512):
        out = torch.empty(blocks * 256, device=dev)
        iters = 4000
        st = VP(torch.cuda.current_stream().cuda_stream)
        lib.exp_mfma_f32(VP(srcf.data_ptr()), VP(out.data_ptr()), blocks, 10, st)
        torch.cuda.synchronize()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        lib.exp_mfma_f32(VP(srcf.data_ptr()), VP(out.data_ptr()), blocks, iters, st)
        b.record()
        b.synchronize()
        ms = a.elapsed_time(b)
        mfmas = blocks * 4 * iters * 8
        flops = mfmas * 32 * 32 * 2 * 2
        res[f"f32_32x32x2_blocks{blocks}"] = {"ms": round(ms, 3), "TFLOPs": round(flops / ms / 1e9, 1)}
        print(f"f32 blocks{blocks}", res[f"f32_32x32x2_blocks{blocks}"], flush=True)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
